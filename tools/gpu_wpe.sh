set -o pipefail
for c in 3 5; do
  timeout -k 10 300 python -u tools/perf.py --config $c --rounds 2 --reps 2 cadence_amd/libcdr.so variants/libcdr_wpe4.so > gpurun_out/r1t_c${c}.log 2>&1 || exit $?
  grep -o '"lib": "[^"]*", "median_ms": [0-9.]*' gpurun_out/r1t_c${c}.log
done
