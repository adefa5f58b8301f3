#!/bin/bash
# One launcher for the GPU-box runs (through gpurun): every GPU step under its own time limit,
# steps chained so the first failure ends the run, outputs under gpurun_out/<tag>/.
#
#   tools/gpu.sh tests    <tag> [test files...]   the -m gpu suite (or a subset) + smoke()
#   tools/gpu.sh pmc      <tag>                   PMC traffic of the C2-C5 steps and C2 --tasks
#                                                 (profiles/traffic_*.json, keyed by libcdr.so's SHA-1)
#   tools/gpu.sh bench    <tag>                   the bench lines: C2 (CPU baseline + rocprofv3 kernel
#                                                 stats of the same command), C3-C5, configs[3] at the
#                                                 count limit, --tasks C2/C3/C5
#   tools/gpu.sh lines    <tag>                   the NDC (configs[4]) and carry-in lines (parity in each)
#   tools/gpu.sh kstats   <tag> <configs...>      rocprofv3 kernel stats of C<n> steps
#   tools/gpu.sh ab       <tag> <B> <configs...>  A/B step times: libcdr.so vs B (variant name or
#                                                 env:VAR=value), A B A B per config
#   tools/gpu.sh perfab   <tag> "<cfgs>" <libs>  interleaved in-process A/B of libcdr.so vs variant libs
#                                                 (tools/perf.py; PERF_ARGS adds its flags)
#   tools/gpu.sh multirank <tag>                  bench.py's multi-rank path, ranks sharing the GPU
#   tools/gpu.sh ingest   <tag>                   on-device thriftrw decode -> replay (tools/ingest_bench.py)
#   tools/gpu.sh calib    calib                   PMC calibration kernels (tools/calib.hip built into
#                                                 tools/build/calib; summarise with tools/calib.py)
set -o pipefail
task=$1; tag=${2:-$1}; shift 2 2>/dev/null || shift $#
out=gpurun_out/$tag; mkdir -p "$out"
export TMPDIR=/tmp
sha1sum cadence_amd/libcdr.so > "$out/lib_sha1"
B="timeout -k 10"

bench_line() {  # name limit args...
  local name=$1 lim=$2; shift 2
  $B "$lim" python -u bench.py "$@" > "$out/$name.json" 2> "$out/$name.log" || { tail -20 "$out/$name.log"; return 1; }
  tail -c 400 "$out/$name.json"; echo
}

case $task in
  tests)
    $B 1000 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 \
      || { tail -30 "$out/tests.log"; exit 1; }
    tail -2 "$out/tests.log"
    $B 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
    tail -1 "$out/smoke.log" ;;
  pmc)
    bash tools/pmc.sh ${tag}c2 cadence_amd/libcdr.so --config 2 > "$out/pmc_c2.log" 2>&1 || exit 1
    python3 tools/traffic.py ${tag}c2 C2-1000000wf-sliced ${tag}_c2 k_replay_fast > "$out/traffic_c2.log" 2>&1 || exit 1
    for c in 3 4 5; do
      bash tools/pmc.sh ${tag}c$c cadence_amd/libcdr.so --config $c > "$out/pmc_c$c.log" 2>&1 || exit 1
      python3 tools/traffic.py ${tag}c$c C$c-1000000wf-sliced ${tag}_c$c k_replay k_tables > "$out/traffic_c$c.log" 2>&1 || exit 1
    done
    bash tools/pmc.sh ${tag}t2 cadence_amd/libcdr.so --config 2 --tasks > "$out/pmc_t2.log" 2>&1 || exit 1
    python3 tools/traffic.py ${tag}t2 C2-1000000wf-sliced-tasks ${tag}_c2_tasks k_replay_fast > "$out/traffic_t2.log" 2>&1 || exit 1
    cp profiles/traffic_C*-1000000wf-sliced*.json "$out/" && echo "pmc set done" ;;
  bench)
    bench_line bench_c2 400 || exit 1
    $B 300 rocprofv3 --kernel-trace --stats -d "$out/prof_c2" -o run -- python3 bench.py --steps 20 --warmup 5 \
      --no-cpu-baseline --no-parity --no-refresh --no-stream-peak --no-host-path > "$out/prof_c2.json" 2> "$out/prof_c2.log" || exit 1
    for c in 3 4 5; do bench_line bench_c$c 400 --config $c --no-stream-peak || exit 1; done
    bench_line bench_c4_long 400 --config 4 --long-stride 125000 --no-cpu-baseline --no-stream-peak --no-refresh || exit 1
    bench_line bench_c2_tasks 400 --tasks --steps 10 --warmup 2 --no-refresh --no-stream-peak || exit 1
    bench_line bench_c3_tasks 400 --tasks --config 3 --steps 10 --warmup 2 --no-refresh --no-stream-peak || exit 1
    bench_line bench_c5_tasks 400 --tasks --config 5 --steps 10 --warmup 2 --no-refresh --no-stream-peak || exit 1
    echo "bench set done" ;;
  lines)
    bench_line ndc_forks_1m 600 --ndc-forks --wfs 1000000 --steps 5 --warmup 1 || exit 1
    for c in 3 5; do bench_line carry_c$c 600 --carry --config $c --wfs 1000000 --steps 10 --warmup 2 || exit 1; done
    bench_line carry_tasks_c3 600 --carry --tasks --config 3 --wfs 1000000 --steps 10 --warmup 2 || exit 1 ;;
  kstats)
    for c in "$@"; do
      $B 300 rocprofv3 --kernel-trace --stats -d "$out/c$c" -o run -- python3 bench.py --config $c --steps 10 --warmup 3 \
        --no-cpu-baseline --no-parity --no-refresh --no-host-path > "$out/c$c.json" 2> "$out/c$c.log" || exit 1
    done ;;
  ab)
    b=$1; shift
    if [[ $b == env:* ]]; then benv=${b#env:}; else benv=CDR_LIB=variants/libcdr_$b.so; fi
    flags="--steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-refresh --no-host-path --no-stream-peak $BENCH_ARGS"
    for c in "$@"; do
      for r in 1 2; do
        env $AENV $B 300 python bench.py --config $c $flags > "$out/c${c}_A$r.json" 2> "$out/c${c}_A$r.log" || exit 1
        env $benv $B 300 python bench.py --config $c $flags > "$out/c${c}_B$r.json" 2> "$out/c${c}_B$r.log" || exit 1
      done
    done
    python3 - "$out" <<'EOF'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c*_[AB]*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.rsplit("/", 1)[1], f"{d['ms_per_step']:.3f} ms/step kernel {d['roofline']['kernel_ms']:.3f} ms")
EOF
    ;;
  perfab)  # interleaved in-process A/B (tools/perf.py) per config: perfab <tag> "<configs>" <libs...>
    cfgs=$1; shift
    for c in $cfgs; do
      $B 400 python -u tools/perf.py --config $c --rounds 4 $PERF_ARGS cadence_amd/libcdr.so "$@" > "$out/c$c.log" 2>&1 \
        || { tail "$out/c$c.log"; exit 1; }
      echo "C$c"; grep '"lib"' "$out/c$c.log"
    done ;;
  multirank)
    export CDR_BENCH_BACKEND=gloo
    $B 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
      bench.py --gpus 2 --wfs 300000 --steps 5 --warmup 2 --no-cpu-baseline --no-refresh --no-stream-peak \
      > "$out/c2_n2.json" 2> "$out/c2_n2.log" || exit 1
    $B 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 \
      bench.py --gpus 4 --config 4 --wfs 100000 --steps 3 --warmup 1 --no-cpu-baseline --no-refresh --no-stream-peak \
      > "$out/c4_n4.json" 2> "$out/c4_n4.log" || exit 1 ;;
  ingest)
    for c in 2 3 5; do
      $B 300 python tools/ingest_bench.py --config $c --wfs ${WFS:-200000} > "$out/c$c.json" 2> "$out/c$c.err" || exit 1
    done
    cat "$out"/c*.json ;;
  calib)
    bin=tools/build/calib
    $B 120 $bin 2 > "$out/plain.log" 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- $bin 2 > "$out/fetch.log" 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- $bin 2 > "$out/write.log" 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$out/rdreq" -o run -- $bin 2 > "$out/rdreq.log" 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$out/wrreq" -o run -- $bin 2 > "$out/wrreq.log" 2>&1 ;;
  *)
    sed -n '2,20p' "$0"; exit 2 ;;
esac
