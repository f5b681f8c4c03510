# Headline bench under tail-kernel launch knobs (tile depth NLS_KZ_FUSED, XCD-banded
# tile order NLS_TILE_REMAP, grid multiplier NLS_GRID_MULT), same box, two rounds.
# usage: bash tools/tail_sweep.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tail_sweep
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 6 --warmup 2 --prof-steps 4 --no-cpu-baseline \
    > gpurun_out/tail_sweep/$tag.json 2> gpurun_out/tail_sweep/$tag.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/tail_sweep/$tag.json'));k=d['step_roofline']['gpu_kernel_ms_per_step'];print('$tag',round(d['ms_per_step'],3),'tail',round(k['final'],3),'upd',round(k['update'],3))"
}
# round-2 first sweep (two tiles per workgroup by default then): base, kz 8/16/64,
# remap, grid x32; second sweep (one tile per workgroup, the default since): tile depths
for r in 1 2; do
  run base$r NLS_DUMMY=0
  run kz8_$r NLS_KZ_FUSED=8
  run kz16_$r NLS_KZ_FUSED=16
  run kz64_$r NLS_KZ_FUSED=64
  run kz128_$r NLS_KZ_FUSED=128
done
