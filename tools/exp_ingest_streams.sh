for k in 1 2 4 1 2 4; do
  timeout -k 10 120 python3 bench.py --no-cpu --sustain 0 --steps 30 --ingest-steps 100 --ingest-streams $k > gpurun_out/ing_$k.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/ing_$k.json').read().strip().splitlines()[-1]); i=d['ingest']; print('streams', $k, i['frames_per_s'], i['h2d_GBs_per_gpu'], i['bit_exact'], d['value'])"
done
