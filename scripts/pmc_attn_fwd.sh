set -o pipefail
mkdir -p gpurun_out/r5/pmc_fwd
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/r5/pmc_fwd/new -o p -- python3 $R/benchmarks/probes/attn_one.py --iters 3 --which fwd > $R/gpurun_out/r5/pmc_fwd/new.log 2>&1 || exit 1
DPH_ATTN_FWD=legacy timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/r5/pmc_fwd/old -o p -- python3 $R/benchmarks/probes/attn_one.py --iters 3 --which fwd > $R/gpurun_out/r5/pmc_fwd/old.log 2>&1 || exit 1
C2="SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC"
timeout -s KILL 90 rocprofv3 --pmc $C2 -d $R/gpurun_out/r5/pmc_fwd/new2 -o p -- python3 $R/benchmarks/probes/attn_one.py --iters 3 --which fwd > $R/gpurun_out/r5/pmc_fwd/new2.log 2>&1 || exit 1
DPH_ATTN_FWD=legacy timeout -s KILL 90 rocprofv3 --pmc $C2 -d $R/gpurun_out/r5/pmc_fwd/old2 -o p -- python3 $R/benchmarks/probes/attn_one.py --iters 3 --which fwd > $R/gpurun_out/r5/pmc_fwd/old2.log 2>&1 || exit 1
for x in new old new2 old2; do f=$(ls $R/gpurun_out/r5/pmc_fwd/$x/*/*.db $R/gpurun_out/r5/pmc_fwd/$x/*.db 2>/dev/null | head -1); echo "== $x $f"; python3 $R/benchmarks/pmc_summary.py "$f" --match attn_fwd; done > $R/gpurun_out/r5/pmc_fwd/summary.txt 2>&1
