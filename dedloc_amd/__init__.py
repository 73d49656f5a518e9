"""dedloc_amd — MI355X-native collaborative training (DeDLOC capabilities, re-designed for CDNA4).

Subpackages: ``ops`` (HIP kernels via torch.library), ``models`` (ALBERT, SwAV ResNet-50),
``optim`` (fused LAMB/LARC, CollaborativeOptimizer), ``averaging`` (butterfly all-reduce over RCCL),
``dht`` (native control-plane DHT), ``training`` (peer loops), ``cli`` (reference entry points),
``emulation`` (heterogeneity/churn), ``data`` (synthetic WikiText/ImageNet streams).
"""
__version__ = "0.1.0"
