"""MI355X-native CTR training hot path of jqsl2012/RL_CTR_Prediction.

FM / FFM / DeepFM / InnerPNN / Feature_Embedding / PolicyGradient with the reference's construction API,
running on hand-written gfx950 HIP kernels behind the C ABI in include/ctr_hip.h
(libctr_hip.so). See DESIGN.md.
"""
from .feature_embedding import Feature_Embedding
from .ffm_trainer import FusedFFMTrainer
from .optim import DenseAdam
from .p_model import FFM, FM, DeepFM, InnerPNN
from .pg_model import Net, PolicyGradient
from .sharded import ShardedCTRTrainer
from .trainer import FusedCTRTrainer

__all__ = ["FM", "FFM", "DeepFM", "InnerPNN", "Feature_Embedding", "Net", "PolicyGradient", "FusedCTRTrainer",
           "FusedFFMTrainer", "ShardedCTRTrainer", "DenseAdam"]
