set -o pipefail
for L in oldsort newsort; do
for c in 3 5; do
CDR_LIB=variants/libcdr_$L.so timeout -k 10 400 python -u tools/perf.py --config $c --wfs 1000000 --rounds 2 --reps 2 --no-wave variants/libcdr_$L.so > gpurun_out/r1p_${L}_c$c.log 2>&1 || exit $?
echo "$L c$c $(grep '{' gpurun_out/r1p_${L}_c$c.log)"
done; done
