set -o pipefail
for c in 3 5 4; do
  timeout -k 10 300 python -u tools/perf.py --config $c --rounds 2 --reps 2 --wave-all cadence_amd/libcdr.so > gpurun_out/r1q_c${c}_waveall.log 2>&1 || exit $?
  echo "c$c wave-all $(grep -o '"median_ms": [0-9.]*' gpurun_out/r1q_c${c}_waveall.log)"
  for lim in 6,10,8,512 4,8,4,256 12,16,16,1024 8,12,8,2048; do
    CDR_LANE_MAX=$lim timeout -k 10 300 python -u tools/perf.py --config $c --rounds 2 --reps 2 cadence_amd/libcdr.so > gpurun_out/r1q_c${c}_$lim.log 2>&1 || exit $?
    echo "c$c lanes<=$lim $(grep -o '"median_ms": [0-9.]*' gpurun_out/r1q_c${c}_$lim.log)"
  done
done
