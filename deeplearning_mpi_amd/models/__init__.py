from .engine import EngineModule  # noqa: F401
from .resnet import ARCHS, ResNet, resnet18, resnet34, resnet50, resnet101, resnet152  # noqa: F401
from .unet import UNet  # noqa: F401
