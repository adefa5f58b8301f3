set -o pipefail
mkdir -p gpurun_out/depth
for c in 3 5; do
timeout -k 10 300 python -u tools/perf.py --config $c --rounds 3 --reps 3 variants/libcdr_base.so variants/libcdr_d1p1.so variants/libcdr_d1p4.so variants/libcdr_d2p4.so variants/libcdr_d2p4w3.so variants/libcdr_d1p4w3.so > gpurun_out/depth/c$c.json 2>gpurun_out/depth/c$c.err || exit 1
cat gpurun_out/depth/c$c.json
done
