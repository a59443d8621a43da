"""Binned iteration and DataLoader length (lddl/torch/dataloader.py:32-105).

`Binned` picks, for every step, one bin with `random.choices(range(n_bins),
weights=samples_remaining)` on a world-identical state (seeded with base_seed + epoch), so all
ranks draw their step's batch from the same bin."""
import torch

from ..random import choices, seeded_state
from .datasets import ParquetDataset


class Binned:
    def __init__(self, dataloaders, base_seed=12345, start_epoch=0, logger=None):
        self._dataloaders = dataloaders
        self._base_seed = base_seed
        self._epoch = start_epoch - 1
        self._logger = logger
        self._world_rng_state = None

    def __len__(self):
        return sum(len(dl) for dl in self._dataloaders)

    def _get_batch_size(self, batch):
        raise NotImplementedError('Binned is an abstract class!')

    def _choices(self, population, weights=None, cum_weights=None, k=1):
        c, self._world_rng_state = choices(population, weights=weights, cum_weights=cum_weights,
                                           k=k, rng_state=self._world_rng_state)
        return c

    def __iter__(self):
        self._epoch += 1
        self._world_rng_state = seeded_state(self._base_seed + self._epoch)
        remaining = [len(dl.dataset) for dl in self._dataloaders]
        its = [iter(dl) for dl in self._dataloaders]
        for i in range(len(self)):
            b = self._choices(list(range(len(its))), weights=remaining, k=1)[0]
            if self._logger is not None:
                self._logger.to('rank').info('{}-th iteration selects bin_id = {}'.format(i, b))
            assert remaining[b] > 0
            batch = next(its[b])
            remaining[b] -= self._get_batch_size(batch)
            yield batch
        assert sum(remaining) == 0


class DataLoader(torch.utils.data.DataLoader):
    """Length = batches the workers really produce: every worker ends with a partial batch."""

    def __len__(self):
        if isinstance(self.dataset, ParquetDataset):
            nw = max(self.num_workers, 1)
            files_per_worker = self.dataset.num_files_per_rank // nw
            per_worker = self.dataset.num_samples_per_file * files_per_worker
            return ((per_worker - 1) // self.batch_size + 1) * nw
        return super().__len__()
