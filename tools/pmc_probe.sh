# One rocprofv3 PMC pass over tools/gemm_split_probe <paths> (kernel names carry the variant), summarised per
# kernel into gpurun_out/pmc_probe_<tag>.txt: wave-cycle split, MFMA busy, LDS stalls / conflicts, clock.
#   gpurun -- 'bash tools/pmc_probe.sh <tag> x2ppwxn x2ppwxw ...'
set -o pipefail
TAG=${1:?tag}; shift
R=$PWD
export TMPDIR=/tmp
RAW=/tmp/pmc_probe_$TAG
mkdir -p $RAW gpurun_out
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $RAW -o run -- \
    $R/tools/gemm_split_probe "$@" > $R/gpurun_out/pmc_probe_$TAG.log 2>&1 && \
python3 $R/tools/pmc_probe_summary.py $RAW > $R/gpurun_out/pmc_probe_$TAG.txt
rc=$?
rm -rf $RAW
cat $R/gpurun_out/pmc_probe_$TAG.txt
exit $rc
