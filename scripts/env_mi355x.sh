#!/usr/bin/env bash
# Environment for one 8x MI355X node (xGMI fully connected): source this before launching.
# Replaces the reference's Slingshot/NCCL/MPICH block (README.md:198-210, docs/guide/nccl_tuning.md,
# every scripts/**/run_*.sh): none of the FI_CXI_*, NCCL_SOCKET_IFNAME=hsn, AWS-OFI or MPICH_GPU_* knobs apply
# inside an xGMI node.  Defaults below are conservative; sweep the commented ones with benchmarks/comm_bench.py.

# dmabuf-based IPC (the only mode the host driver supports; RCCL / CUDA-tensor sharing fails without it)
export HSA_ENABLE_IPC_MODE_LEGACY=0
# one OpenMP thread per rank unless the data pipeline needs more
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}
# surface collective mismatches / hangs instead of blocking forever (PyTorch c10d watchdog, applies to RCCL)
export TORCH_NCCL_ASYNC_ERROR_HANDLING=${TORCH_NCCL_ASYNC_ERROR_HANDLING:-1}
export TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC=${TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC:-600}
# RCCL logging: VERSION prints the library version once; INFO/TRACE + NCCL_DEBUG_SUBSYS=INIT,COLL,P2P to debug
export NCCL_DEBUG=${NCCL_DEBUG:-VERSION}

# ---- knobs to sweep on the box (leave unset for RCCL's own topology-aware defaults) ----
# benchmarks/rccl_sweep.py measures them and writes the winning exports for bucket-sized traffic; picked up here
# when present (DPH_RCCL_ENV overrides the path) and measured at this job's rank count (DPH_NPROC, default 8);
# the file only fills knobs the user left unset
_dph_rccl_env=${DPH_RCCL_ENV:-$(dirname "${BASH_SOURCE[0]}")/../results/rccl_sweep/rccl_env.sh}
if [ -f "$_dph_rccl_env" ]; then
  _dph_sweep_n=$(sed -n 's/^DPH_RCCL_SWEEP_NPROC=//p' "$_dph_rccl_env")
  if [ "${_dph_sweep_n:-0}" = "${DPH_NPROC:-8}" ]; then
    . "$_dph_rccl_env"
  else
    echo "env_mi355x.sh: ignoring $_dph_rccl_env (swept at ${_dph_sweep_n:-?} ranks, job has ${DPH_NPROC:-8})" >&2
  fi
fi
unset _dph_rccl_env _dph_sweep_n
# export NCCL_MIN_NCHANNELS=32          # more channels -> more xGMI links busy per collective
# export NCCL_MAX_NCHANNELS=64
# export NCCL_ALGO=Ring                 # Ring | Tree (direct/one-shot variants are chosen by RCCL per size)
# export NCCL_PROTO=Simple              # LL | LL128 | Simple
# export RCCL_MSCCL_ENABLE=1            # MSCCL algorithms for small all-reduce / all-gather
# export RCCL_MSCCLPP_ENABLE=1
# export NCCL_P2P_NET_CHUNKSIZE=524288

# ---- debugging aids ----
# export AMD_SERIALIZE_KERNEL=3         # serialise kernel launches (HIP analogue of CUDA_LAUNCH_BLOCKING=1)
# export HIP_LAUNCH_BLOCKING=1
# export TORCH_DISTRIBUTED_DEBUG=DETAIL # check collective shapes / order across ranks
# export DPH_KERNELS=aten               # run the stock PyTorch-ROCm ops instead of the HIP kernels (parity runs)
