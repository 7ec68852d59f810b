#!/usr/bin/env bash
# Same-box A/B of the poly-mul: whole-plane VALU kernel (RNT_PLANE=3) vs the
# MFMA kernel (RNT_PLANE=5), then the NTT workload and a kernel trace of the
# MFMA poly-mul.  Outputs under gpurun_out/r04/.
set -euo pipefail
O=gpurun_out/r04
mkdir -p $O
for rep in 1 2; do
  RNT_PLANE=3 timeout -k 10 240 python bench.py --no-cpu-baseline > $O/ab_plane3_$rep.json 2> $O/ab_plane3_$rep.err
  RNT_PLANE=5 timeout -k 10 240 python bench.py --no-cpu-baseline > $O/ab_plane5_$rep.json 2> $O/ab_plane5_$rep.err
done
RNT_PLANE=5 timeout -k 10 240 python bench.py --no-cpu-baseline --no-power --workload ntt > $O/ntt_plane5.json 2> $O/ntt_plane5.err
RNT_PLANE=3 timeout -k 10 240 python bench.py --no-cpu-baseline --no-power --workload ntt > $O/ntt_plane3.json 2> $O/ntt_plane3.err
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
RNT_PLANE=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mf -o mf -- python bench.py --no-cpu-baseline --no-power --steps 5 --warmup 2 > $O/prof_mf.json 2> $O/prof_mf.err
