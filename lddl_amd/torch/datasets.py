"""Parquet streaming datasets (lddl/torch/datasets.py:46-286), same sample order as the reference:

* file counts from `.num_samples.json` (or parquet footers), strided over ranks and summed with
  all_reduce (RCCL under nccl) (`_get_files`, 161-201);
* per epoch a world-identical permutation of the files (`random.sample` on a state seeded with
  base_seed + epoch), then `files[rank::world][worker::num_workers]` (247-272);
* a shuffle buffer per worker (46-109): once warm, each incoming sample replaces a random slot
  (`randrange` on a state seeded with base_seed + (epoch * world + rank) * workers + worker) whose
  old occupant is yielded; the tail is shuffled.
Every rank yields num_samples_per_file * files_per_rank samples (files hold N or N+1 samples
after load balancing; the +1 is dropped). The reference asserts min + 1 == max and so fails on
perfectly balanced shards; this build accepts max - min <= 1.
"""
import json
import os

import pyarrow.parquet as pq
import torch
from torch.utils.data import IterableDataset, get_worker_info

from ..random import randrange, sample, seeded_state, shuffle
from ..types import File
from ..utils import get_num_samples_of_parquet
from .utils import get_nproc_per_node, get_num_nodes, get_node_rank, get_rank, get_world_size


class ShuffleBuffer:
    def __init__(self, files, max_num_samples_to_yield, decode_record_batch, size,
                 warmup_factor, logger, rng_state):
        wasted = sum(f.num_samples for f in files) - max_num_samples_to_yield
        assert 0 <= wasted <= len(files)
        self._files = files
        self._max = max_num_samples_to_yield
        self._decode = decode_record_batch
        self._size = size
        self._warmup = warmup_factor
        self._logger = logger
        self._rng_state = rng_state

    @property
    def num_samples(self):
        return sum(f.num_samples for f in self._files)

    def _randrange(self, stop):
        n, self._rng_state = randrange(stop, rng_state=self._rng_state)
        return n

    def __iter__(self):
        buf = []
        to_yield = min(self._max, self.num_samples)
        remaining = to_yield
        for f in self._files:
            self._logger.to('worker').info('Reading {}'.format(f.path))
            # one thread per reader: the loader runs one reader per DataLoader worker, and
            # pyarrow's default pool (os.cpu_count() threads in every worker) oversubscribes
            # the host's granted CPUs and throttles the training process
            for b in pq.read_table(f.path, use_threads=False).to_batches():
                for s in self._decode(b):
                    if remaining <= 0:
                        return
                    if len(buf) >= min(self._size, (to_yield - remaining + 1) * self._warmup):
                        k = self._randrange(len(buf))
                        yield buf[k]
                        buf[k] = s
                        remaining -= 1
                    else:
                        buf.append(s)
        self._rng_state = shuffle(buf, rng_state=self._rng_state)
        for s in buf:
            if remaining <= 0:
                return
            yield s
            remaining -= 1


def _identity(x):
    return x


class ParquetDataset(IterableDataset):
    def __init__(self, file_paths, transform=_identity, local_rank=0, shuffle_buffer_size=16384,
                 shuffle_buffer_warmup_factor=16, base_seed=12345, logger=None, start_epoch=0):
        super().__init__()
        self._transform = transform
        self._local_rank = local_rank
        self._shuffle_buffer_size = shuffle_buffer_size
        self._shuffle_buffer_warmup_factor = shuffle_buffer_warmup_factor
        self._base_seed = base_seed
        self._rank = get_rank()
        self._world_size = get_world_size()
        self._nproc_per_node = get_nproc_per_node(local_rank)
        self._num_nodes = get_num_nodes(nproc_per_node=self._nproc_per_node)
        self._node_rank = get_node_rank(nproc_per_node=self._nproc_per_node)
        self._epoch = start_epoch - 1
        self._logger = logger
        assert len(file_paths) % self._num_nodes == 0
        assert len(file_paths) % self._world_size == 0
        self._files = self._get_files(file_paths)
        hi = max(f.num_samples for f in self._files)
        lo = min(f.num_samples for f in self._files)
        assert hi - lo <= 1, 'files are not load balanced ({}..{} samples)'.format(lo, hi)
        self._num_samples_per_file = lo
        total = sum(f.num_samples for f in self._files)
        lost = total - lo * len(self._files)
        self._logger.to('node').warning('lost {}/{}={}% samples in total'.format(
            lost, total, lost / max(total, 1) * 100))
        self._world_rng_state = None
        self._worker_rng_state = None

    def _get_files(self, file_paths):
        counts = torch.zeros(len(file_paths), dtype=torch.long)
        if self._world_size > 1 and torch.distributed.get_backend() == 'nccl':
            counts = counts.to('cuda')
        cache = {}
        for i in range(self._rank, len(file_paths), self._world_size):
            fp = file_paths[i]
            dn, bn = os.path.dirname(fp), os.path.basename(fp)
            if dn not in cache:
                try:
                    with open(os.path.join(dn, '.num_samples.json')) as f:
                        cache[dn] = json.load(f)
                except Exception as e:
                    self._logger.to('rank').warning('failed to load {}: {}'.format(
                        os.path.join(dn, '.num_samples.json'), e))
                    cache[dn] = None
            if cache[dn] is not None and bn in cache[dn]:
                counts[i] = cache[dn][bn]
            else:
                counts[i] = get_num_samples_of_parquet(fp)
        if self._world_size > 1:
            torch.distributed.all_reduce(counts, op=torch.distributed.ReduceOp.SUM)
        return [File(fp, n) for fp, n in zip(file_paths, counts.tolist())]

    def __len__(self):
        return self._num_samples_per_file * len(self._files) // self._world_size

    @property
    def num_samples_per_file(self):
        return self._num_samples_per_file

    @property
    def num_files_per_rank(self):
        return len(self._files) // self._world_size

    def _decode_record_batch(self, b):
        raise NotImplementedError('ParquetDataset is an abstract/interface class!')

    def _init_worker(self):
        info = get_worker_info()
        nw, wr = (1, 0) if info is None else (info.num_workers, info.id)
        assert len(self._files) % (self._world_size * nw) == 0
        self._logger.init_for_worker(wr)
        return wr, nw

    def _init_rng_states(self, worker_rank, num_workers):
        self._world_rng_state = seeded_state(self._base_seed + self._epoch)
        self._worker_rng_state = seeded_state(
            self._base_seed + (self._epoch * self._world_size + self._rank) * num_workers +
            worker_rank)

    def __iter__(self):
        self._epoch += 1
        wr, nw = self._init_worker()
        self._init_rng_states(wr, nw)
        files, self._world_rng_state = sample(self._files, len(self._files),
                                              rng_state=self._world_rng_state)
        self._logger.to('node').warning('epoch = {}'.format(self._epoch))
        worker_files = files[self._rank::self._world_size][wr::nw]
        sb = ShuffleBuffer(worker_files, self._num_samples_per_file * len(worker_files),
                           self._decode_record_batch, self._shuffle_buffer_size,
                           self._shuffle_buffer_warmup_factor, self._logger,
                           self._worker_rng_state)
        for s in sb:
            yield self._transform(s)
