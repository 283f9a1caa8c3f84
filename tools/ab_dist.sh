#!/bin/bash
# N>1 path at world 1 on one box: the bench at N=1 (no collective) against --dist with
# liborbamd's RCCL communicator (ncclAllGather on graph 0's stream / on the exchange's own stream) and against
# torch's ProcessGroupNCCL, interleaved rounds; then one kernel trace of the rccl form for the queue map.
# usage: tools/ab_dist.sh <tag> [rounds]
T=$1; R=${2:-3}
mkdir -p gpurun_out
summ='import sys,json; d=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith("{")][-1]); print("%.0f bit_exact=%s exch=%.3f ag=%.4f %s" % (d["value"], d["bit_exact"], d["stage_ms_per_step"].get("exchange",0), d["stage_ms_per_step"].get("allgather",0), d["collective"][:60]))'
common="--steps 200 --warmup 20 --no-cpu --sustain 0 --ingest-steps 0"
port=29611
for r in $(seq 1 $R); do
  out=$(timeout -k 10 150 python3 bench.py $common | python3 -c "$summ") || exit $?
  echo "r$r n1:           $out"
  for mode in "rccl graph0" "rccl own" "torch auto"; do
    set -- $mode
    port=$((port+1))
    out=$(timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
          --master-port $port bench.py --dist --collective $1 --exchange-stream $2 $common 2>/dev/null | python3 -c "$summ") || exit $?
    echo "r$r dist $1/$2: $out"
  done
done
# kernel trace of the rccl form (bench.py itself under rocprofv3: WORLD_SIZE etc. from this shell, no launcher)
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((port+1))
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_kt_dist -o kt -- python3 bench.py --dist --steps 20 --warmup 5 \
  --no-cpu --sustain 0 --ingest-steps 0 --no-check > gpurun_out/${T}_kt_dist.log 2>&1 || exit $?
kt=$(find gpurun_out/${T}_kt_dist -name '*kernel_trace.csv' | head -n 1)
python3 tools/queue_map.py "$kt" > gpurun_out/${T}_queue_map_dist.txt && cat gpurun_out/${T}_queue_map_dist.txt
