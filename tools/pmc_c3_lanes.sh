set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r2c_pmc; mkdir -p $out
timeout -k 10 120 python3 tools/perf.py --config 3 --wfs 200000 --rounds 2 --reps 2 --no-wave cadence_amd/libcdr.so > $out/time_lanes.log 2>&1 &&
timeout -k 10 120 python3 tools/perf.py --config 3 --wfs 200000 --rounds 2 --reps 2 --wave-all cadence_amd/libcdr.so > $out/time_wave.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $out/sq1 -o run -- python3 tools/perf.py --config 3 --wfs 200000 --rounds 1 --reps 1 --no-wave cadence_amd/libcdr.so > $out/sq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d $out/sq2 -o run -- python3 tools/perf.py --config 3 --wfs 200000 --rounds 1 --reps 1 --no-wave cadence_amd/libcdr.so > $out/sq2.log 2>&1
echo rc=$?
