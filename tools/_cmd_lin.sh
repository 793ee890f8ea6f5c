export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/lin_probe.py --model pythia-12b --prompts 12 --kshot 10 --reps 2 > gpurun_out/lin_probe_12b_full.json 2> gpurun_out/lin_probe_12b_full.err || { tail -20 gpurun_out/lin_probe_12b_full.err; exit 1; }
cat gpurun_out/lin_probe_12b_full.json
