"""hetseq_9cme_amd: MI355X-native heterogeneous data-parallel training engine with
HetSeq's capabilities (BERT pre-training, MNIST, NER/EL fine-tuning), built on
PyTorch-ROCm + hand-written gfx950 HIP kernels + RCCL over xGMI."""
__version__ = '0.1.0'
