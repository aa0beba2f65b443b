from .act import Act, pad8  # noqa: F401
from .backend import NativeBackend, RefBackend, make_backend  # noqa: F401
from .losses import (BCEWithLogitsLoss, CrossEntropyLoss, backward, bce_with_logits, cross_entropy,  # noqa: F401
                     dice_per_sample, top1_correct)
