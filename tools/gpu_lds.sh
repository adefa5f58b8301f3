set -o pipefail
timeout -k 10 400 python -u tools/perf.py --config 3 --wfs 200000 --rounds 3 --reps 2 --no-wave cadence_amd/libcdr.so variants/libcdr_a2t6.so variants/libcdr_a3t8.so variants/libcdr_a4t10.so variants/libcdr_a8t10.so > gpurun_out/r1o_c3.log 2>&1 || exit $?
grep "{" gpurun_out/r1o_c3.log
timeout -k 10 400 python -u tools/perf.py --config 3 --wfs 200000 --rounds 3 --reps 2 cadence_amd/libcdr.so > gpurun_out/r1o_c3w.log 2>&1 || exit $?
grep "{" gpurun_out/r1o_c3w.log
timeout -k 10 400 python -u tools/perf.py --config 5 --wfs 200000 --rounds 3 --reps 2 --no-wave cadence_amd/libcdr.so variants/libcdr_a2t6.so variants/libcdr_a3t8.so variants/libcdr_a4t10.so variants/libcdr_a8t10.so > gpurun_out/r1o_c5.log 2>&1 || exit $?
grep "{" gpurun_out/r1o_c5.log
