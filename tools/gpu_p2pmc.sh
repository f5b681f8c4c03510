# PMC read/write bytes of the two-vector passes (one counter per pass)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_p2
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  NLS_PASS2=1 NLS_P2_KZ=256 timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/p2_probe.py 512 16 2 > $OUT/p$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, collections, glob, re
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_p2/p*/*counter_collection.csv") + glob.glob("gpurun_out/pmc_p2/p*/*/*counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void nls::", "")
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
cells = 512**3
for k, d in sorted(agg.items()):
    c = {n: sum(v)/len(v) for n, v in d.items()}
    rd = 2*c.get("FETCH_SIZE", 0)*1024; wr = c.get("WRITE_SIZE", 0)*1024
    h, mi = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    print(f"{k[:40]:40s} rd {rd/cells:7.1f} B/cell  wr {wr/cells:6.1f} B/cell  L2hit {h/max(h+mi,1):.2f}")
PY
