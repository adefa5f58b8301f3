set -o pipefail
for c in 3 5; do
timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-stream-peak --no-wave > gpurun_out/r1n_c${c}_lanes.log 2>&1 || exit $?
grep '^{' gpurun_out/r1n_c${c}_lanes.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("%.3g ev/s kernel %.2f ms" % (d["value"], r["kernel_ms"]))'
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1n_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r1n_gpu.log; exit $rc
