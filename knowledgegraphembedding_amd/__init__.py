"""knowledgegraphembedding_amd — MI355X-native KGE scoring / training / ranking path.

Drop-in for kahrabian/KnowledgeGraphEmbedding's KGEModel / TrainDataset /
TestDataset / run.py API; the hot path runs in hand-written HIP kernels for
gfx950 (libkge_hip.so, C-ABI in include/kge_hip.h).
"""
from .dataloader import BidirectionalOneShotIterator, TestDataset, TrainDataset  # noqa: F401
from .model import KGEModel  # noqa: F401
from .optim import KGEAdam  # noqa: F401

__all__ = ["KGEModel", "TrainDataset", "TestDataset", "BidirectionalOneShotIterator", "KGEAdam"]
