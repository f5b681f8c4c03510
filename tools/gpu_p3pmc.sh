# PMC diagnostics of the s-step passes (k_p3d vs k_p2d): wave-state cycles, LDS, HBM bytes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_p3
mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/p2_probe.py 512 16 1 > $OUT/p$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, collections, glob, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_p3/p*/*counter_collection.csv") + glob.glob("gpurun_out/pmc_p3/p*/*/*counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void nls::", "")
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
cells = 512**3
for k, d in sorted(agg.items()):
    if "p2d" not in k and "p3d" not in k and "tail" not in k:
        continue
    c = {n: sum(v)/len(v) for n, v in d.items()}
    rd = 2*c.get("FETCH_SIZE", 0)*1024; wr = c.get("WRITE_SIZE", 0)*1024
    wc = c.get("SQ_WAVE_CYCLES", 1)
    print(f"{k[:34]:34s} rd {rd/cells:6.1f} wr {wr/cells:5.1f} B/cell | wait {c.get('SQ_WAIT_ANY',0)/wc:.2f} "
          f"instwait {c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} active {c.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
          f"ldswait {c.get('SQ_WAIT_INST_LDS',0)/wc:.2f} | lds bank {c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_LDS_IDX_ACTIVE',1),1):.2f} "
          f"lds_active {c.get('SQ_LDS_IDX_ACTIVE',0):.3g} insts_lds {c.get('SQ_INSTS_LDS',0):.3g} wavecyc {wc:.3g}")
PY
