# same-box A/B: lib (A) vs lib_v (B), alternating probes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do for v in lib lib_v; do
  echo "== $v" ; NLS_AMD_LIB=$PWD/nonlinear-solvers_amd/$v/libnls_amd.so timeout -k 10 120 python tools/p2_probe.py ${N:-512} 16 4 || exit 1
done; done > gpurun_out/p2ab.log 2>&1
python - <<'PY'
import re
cur=None; res={}
for l in open("gpurun_out/p2ab.log"):
    if l.startswith("=="): cur=l.split()[1]; continue
    m=re.match(r"J=\s*(\d+)\s+([\d.]+) ms", l)
    if m: res.setdefault(cur,{}).setdefault(int(m.group(1)),[]).append(float(m.group(2)))
    m=re.match(r"update per step ([\d.]+)", l)
    if m: res.setdefault(cur,{}).setdefault("upd",[]).append(float(m.group(1)))
for v,d in res.items():
    print(v, {k: [round(x,3) for x in xs] for k,xs in d.items()})
PY
