set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_variant_ab.sh r03d mad 512 base mad mul || exit 1
timeout -k 10 240 tools/ubench gpurun_out/r03d/ubench.jsonl > gpurun_out/r03d/ubench.txt 2>&1 || exit 2
grep "chip" gpurun_out/r03d/ubench.txt | grep -E "mad_u64|mul_lo|xor_shr"
timeout -k 10 300 python -u tools/depth_probe.py 64 > gpurun_out/r03d/depth.txt 2>&1 || exit 3
cat gpurun_out/r03d/depth.txt
