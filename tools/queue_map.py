"""Which hardware queue each HIP stream's kernels landed on, from a rocprofv3 kernel trace
(Stream_Id / Queue_Id columns): one line per stream with its kernel count, the queues it used and its most
frequent kernels. The bench's four graph streams should each own one queue; an idle stream created before them
can push two graph streams onto one queue (profiles/r04_idle_stream_cost.log).

usage: python3 tools/queue_map.py <kernel_trace.csv>
"""
import collections
import csv
import sys


def main(path):
    per = collections.defaultdict(lambda: (collections.Counter(), collections.Counter()))
    for r in csv.DictReader(open(path)):
        q, k = per[r["Stream_Id"]]
        q[r["Queue_Id"]] += 1
        k[r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")] += 1
    for s in sorted(per, key=lambda x: int(x)):
        q, k = per[s]
        print("stream %3s: %6d kernels on queue(s) %s | %s" % (
            s, sum(q.values()), dict(q), ", ".join("%s x%d" % kv for kv in k.most_common(4))))
    streams_per_queue = collections.defaultdict(set)
    for s, (q, _) in per.items():
        for qq in q:
            streams_per_queue[qq].add(s)
    print("queues:", {q: sorted(v, key=int) for q, v in sorted(streams_per_queue.items(), key=lambda x: int(x[0]))})


if __name__ == "__main__":
    main(sys.argv[1])
