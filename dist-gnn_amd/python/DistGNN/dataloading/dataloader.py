"""Seed batching, counterpart of python/DistGNN/dataloading/dataloader.py:4-45."""
import torch

__all__ = ["SeedGenerator"]


class SeedGenerator:
    """Iterates `data` in batches of `batch_size` (optionally reshuffled every epoch on the
    data's device; the last partial batch is kept unless drop_last)."""

    def __init__(self, data: torch.Tensor, batch_size: int, shuffle: bool = False,
                 drop_last: bool = False):
        self.data = data
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.step = 0
        self.last_step = 0

    def _num_batches(self):
        n = self.data.shape[0]
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        if self.shuffle:
            self.data = self.data[torch.randperm(self.data.shape[0], device=self.data.device)]
        self.step = 0
        self.last_step = self._num_batches()
        return self

    def __next__(self):
        if self.step >= self.last_step:
            raise StopIteration
        lo = self.step * self.batch_size
        self.step += 1
        return self.data[lo:lo + self.batch_size]

    def __len__(self):
        return self._num_batches()

    def is_finished(self):
        return self.step >= self.last_step
