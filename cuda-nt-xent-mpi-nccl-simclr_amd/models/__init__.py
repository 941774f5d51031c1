"""SimCLR model family: encoders, projection head, GPU augmentations, LARS and the trainer."""
from .augment import AugmentConfig, simclr_view, two_views  # noqa: F401
from .lars import LARS  # noqa: F401
from .simclr import (  # noqa: F401
    MLPEncoder,
    ProjectionHead,
    ResNetEncoder,
    SimCLR,
    param_groups_for_lars,
    resnet18,
    resnet34,
)
from .trainer import SimCLRTrainer, SyntheticImages, TrainConfig  # noqa: F401
