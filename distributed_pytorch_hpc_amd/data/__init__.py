from .cifar import CIFAR10, CIFARDeviceLoader
from .sampler import DistributedSampler, dp_dataloader
from .synthetic import DeviceBatches, ERA5Dataset, MyTrainDataset, SimpleDataset, TokenDataset

__all__ = ["CIFAR10", "CIFARDeviceLoader", "DistributedSampler", "dp_dataloader", "DeviceBatches", "ERA5Dataset", "MyTrainDataset", "SimpleDataset",
           "TokenDataset"]
