set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1r_gpu.log 2>&1 || { tail -30 gpurun_out/r1r_gpu.log; exit 1; }
tail -1 gpurun_out/r1r_gpu.log
for c in 3 4 5; do
  CDR_SERIAL_KERNELS=1 timeout -k 10 300 python -u tools/perf.py --config $c --rounds 2 --reps 2 cadence_amd/libcdr.so > gpurun_out/r1r_c${c}_serial.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/perf.py --config $c --rounds 2 --reps 2 cadence_amd/libcdr.so > gpurun_out/r1r_c${c}_conc.log 2>&1 || exit $?
  echo "c$c serial $(grep -o '"median_ms": [0-9.]*' gpurun_out/r1r_c${c}_serial.log) concurrent $(grep -o '"median_ms": [0-9.]*' gpurun_out/r1r_c${c}_conc.log)"
done
