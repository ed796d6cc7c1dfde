# r06f: the FP64 candidate list as 64-bit (bound, index) entries (YK_CAND64): parity suite on the
# variant, synced A/B at 512 spp, bench A/B (back-to-back steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_variant_ab.sh r06f cand64 512 base cand64 || exit 1
bash tools/gpu_bench_ab.sh r06f_bench base cand64 || exit 1
