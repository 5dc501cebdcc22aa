#!/bin/bash
# SQ counters of the PnP sweep (one rocprofv3 pass per counter group).
set -u
R=$PWD; mkdir -p gpurun_out/pmc_pnp
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
    --output-format csv -d "$R/gpurun_out/pmc_pnp/sq" -o run -- python3 "$R/bench.py" --workload pnp --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_pnp/sq.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_ANY \
    --output-format csv -d "$R/gpurun_out/pmc_pnp/sq2" -o run -- python3 "$R/bench.py" --workload pnp --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_pnp/sq2.log" 2>&1 || exit 1
python3 - "$R/gpurun_out/pmc_pnp" <<'PY'
import csv,glob,sys,collections
for d in ('sq','sq2'):
    fs=glob.glob(sys.argv[1]+'/'+d+'/**/*counter_collection.csv',recursive=True)
    acc=collections.defaultdict(float); n=collections.Counter()
    for f in fs:
        for r in csv.DictReader(open(f)):
            if 'pnp_verify_pk' not in r['Kernel_Name']: continue
            acc[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
    for k in sorted(acc): print(d, k, acc[k]/max(1,len(set(n.values())) and n[k]) , 'per-dispatch-avg over', n[k])
PY
