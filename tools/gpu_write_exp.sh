set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wr
for v in cadence_amd/libcdr.so variants/libcdr_exp8.so; do
  n=$(basename $v .so)
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wr/$n -o run -- python3 tools/perf.py --rounds 1 --reps 2 $v > gpurun_out/wr/$n.log 2>&1 || exit 1
  tail -1 gpurun_out/wr/$n.log
done
