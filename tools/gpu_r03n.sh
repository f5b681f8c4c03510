#!/bin/bash
# Round 3: SQ stall counters of the two-vector passes (G2 256^3 and the headline 512^3).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sq
i=0
for W in g2_3d_256 nlse3d_512; do
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sq/$W/p$i -o run -- python3 bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/sq/$W.p$i.log 2>&1 || exit $?
done
done
echo ok
