summ='import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d["stage_ms_per_step"]; print("%.0f" % d["value"], " ".join("%s=%.3f" % (k, s[k]) for k in ("pyramid","fast_cells","octree","blur","describe","match")))'
python -c "import torch; print(torch.cuda.Stream.priority_range())"
for r in 1 2 3; do for m in none lead lead1; do
  out=$(timeout -k 10 120 python bench.py --sustain 0 --no-cpu --steps 30 --prio $m | python -c "$summ") || exit $?
  echo "r$r prio=$m: $out"
done; done
