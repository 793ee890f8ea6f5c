# rocprofv3 summary of the default bench command (run on the GPU box from the
# repo root): kernel trace + stats, then one PMC pass each for FETCH_SIZE and
# WRITE_SIZE and one for MFMA busy cycles + wave states; summaries (small) go to gpurun_out/profiles_<tag>/, the raw
# traces are deleted so the merge-back stays under its size cap.
#   gpurun -- 'bash tools/prof_cmd.sh r01b [extra bench args]'
set -o pipefail
TAG=${1:?tag}; shift
R=$PWD
export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg --no-processed-leg --extract 0 --configs= $*"
RAW=/tmp/prof_raw
OUT=$R/gpurun_out/profiles_$TAG
mkdir -p $OUT $RAW
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $RAW/stats -o run -- python3 $B > $OUT/bench.json 2> $OUT/bench.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $RAW/fetch -o run -- python3 $B > $OUT/fetch_bench.json 2> $OUT/fetch.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $RAW/write -o run -- python3 $B > $OUT/write_bench.json 2> $OUT/write.err && \
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $RAW/mfma -o run -- python3 $B > $OUT/mfma_bench.json 2> $OUT/mfma.err && \
python3 $R/tools/prof_summary.py --tag $TAG --stats $RAW/stats --fetch $RAW/fetch --write $RAW/write --mfma $RAW/mfma \
    --bench $OUT/bench.json --cmd "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg --no-processed-leg --extract 0 --configs= $*" \
    --out $OUT > $OUT/summary.log
rc=$?
rm -rf $RAW
cut -c1-300 $OUT/bench.json
tail -3 $OUT/summary.log
exit $rc
