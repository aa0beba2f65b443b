import itertools

import pytest
import torch.utils.data as tud

from deeplearning_mpi_amd.data import DistributedSampler


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,world,shuffle,drop_last", list(itertools.product([1, 7, 10, 50000, 283], [1, 2, 3, 8],
                                                                              [True, False], [True, False])))
def test_matches_torch(n, world, shuffle, drop_last):
    ds = _DS(n)
    if drop_last and n < world:
        return
    for rank in range(world):
        for epoch in (0, 3):
            a = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=7, drop_last=drop_last)
            b = tud.DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=7,
                                       drop_last=drop_last)
            a.set_epoch(epoch)
            b.set_epoch(epoch)
            assert list(a) == list(b)
            assert len(a) == len(b)


def test_bad_rank():
    with pytest.raises(ValueError):
        DistributedSampler(_DS(10), num_replicas=2, rank=2)
