from .datasets import (CIFAR10, CarvanaDataset, CifarTransform, SegmentationDataset,  # noqa: F401
                       SyntheticImages, SyntheticMasks, device_batch)
from .sampler import DistributedSampler  # noqa: F401
from .device import DeviceBatches, DeviceCachedDataset, DeviceImageDataset, image_batch_reference  # noqa: F401
