"""MI355X-native data-parallel CIFAR-10 training framework (capabilities of BaamPark/DistributedDataParallel-Cifar10).

Subpackages:
  models/    NetResDeep (reference model/resnet.py parity)
  runtime/   native engine loader + the fused, graph-captured NetResDeep training step (HIP/CDNA4 kernels)
  parallel/  process-group setup (RCCL), flat-bucket DDP wrapper, distributed sampler
  data/      CIFAR-10 readers, synthetic CIFAR-shaped data, device-resident datasets
  utils/     checkpointing, metrics/logging, GPU utilities, the fp32 oracle used by the tests
  csrc/      C++/HIP sources (built in-tree by build.py into _lib/)
"""
__version__ = "0.1.0"
