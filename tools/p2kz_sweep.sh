# Per-pass times of the two-vector passes at 512^3 m=16 under k_p2d tile depths
# (NLS_P2_KZ; default 256 there: 2048 tiles), same box, two rounds.
# usage: bash tools/p2kz_sweep.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/p2kz
for r in 1 2; do
  for kz in 256 128 64 32; do
    NLS_P2_KZ=$kz timeout -k 10 150 python -u tools/p2_probe.py 512 16 3 > gpurun_out/p2kz/kz${kz}_$r.log 2>&1 || exit 1
    echo "kz=$kz round $r"; cat gpurun_out/p2kz/kz${kz}_$r.log
  done
done
