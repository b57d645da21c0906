"""distributed_pytorch_hpc_amd -- an MI355X-native distributed training framework.

Capabilities of negin513/distributed-pytorch-hpc (DDP, FSDP, TP, SP, 2-D hybrid, PP, and the documented-only
Ulysses / ring attention / domain parallelism), rebuilt for AMD Instinct MI355X (gfx950, CDNA4):
hand-written HIP kernels (csrc/) for the hot ops, RCCL over xGMI for every collective, one process per GPU.

Subpackages:
  ops       CDNA4 kernels with autograd (flash attention, RMSNorm, LayerNorm, RoPE, SwiGLU, GELU, CE, embedding)
  parallel  DDP / FSDP engines, tensor + sequence, pipeline, context (Ulysses / ring), domain parallelism
  comm      autograd collectives, process meshes
  models    Llama-2, ResNet, UNet, ViT, pipeline transformer, toys
  train     fused optimizers, trainer loop
  data      synthetic datasets, dp-aware sampler
  runtime   rank discovery / process-group bootstrap, single-node launcher
  utils     logging, config, checkpointing, profiling, metrics, flat buffers
"""
__version__ = "0.1.0"
