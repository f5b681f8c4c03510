#!/bin/bash
# A/B of env knobs on the non-headline bench workloads, same box, rounds interleaved.
# usage: bash tools/wl_ab.sh "<workloads>" "<cfg1>" "<cfg2>" ...   (cfg: "ENV=V ENV=V" or "default")
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wl_ab
WLS=$1; shift
for r in 1 2; do
  for wl in $WLS; do
    for cfg in "$@"; do
      tag=$(echo "$cfg" | tr ' =' '_-')
      out=gpurun_out/wl_ab/${wl}_${tag}_$r.json
      if [ "$cfg" = default ]; then
        timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 5 --warmup 2 > $out 2>/dev/null || exit 1
      else
        env $cfg timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 5 --warmup 2 > $out 2>/dev/null || exit 1
      fi
      python3 -c "import json;d=json.load(open('$out'));print('$wl', '[$cfg]', round(d['value'],1), round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['step_roofline']['gpu_kernel_ms_per_step'].items() if v})"
    done
  done
done
