"""Per node / rank / worker loggers (lddl/torch/log.py:28-133): logger names
`node-<n>`, `node-<n>_local-<l>`, `node-<n>_local-<l>_worker-<w>`; `to('node')` only logs on
local rank 0 / worker 0, `to('rank')` on worker 0, `to('worker')` everywhere."""
import logging
import os
import pathlib

_FMT = ('LDDL - %(asctime)s - %(filename)s:%(lineno)d:%(funcName)s - %(name)s - %(levelname)s '
        ': %(message)s')


def _name(node_rank, local_rank=None, worker_rank=None):
    n = 'node-{}'.format(node_rank)
    if local_rank is not None:
        n += '_local-{}'.format(local_rank)
        if worker_rank is not None:
            n += '_worker-{}'.format(worker_rank)
    return n


class DummyLogger:
    def _noop(self, *a, **k):
        pass

    debug = info = warning = error = critical = log = exception = _noop


class DatasetLogger:
    def __init__(self, log_dir=None, node_rank=0, local_rank=0, log_level=logging.INFO):
        self._log_dir = log_dir
        self._node_rank = node_rank
        self._local_rank = local_rank
        self._worker_rank = None
        self._log_level = log_level
        if log_dir is not None:
            pathlib.Path(log_dir).mkdir(parents=True, exist_ok=True)
        if local_rank == 0:
            self._create(_name(node_rank))
        self._create(_name(node_rank, local_rank))

    def _create(self, name):
        lg = logging.getLogger(name)
        if not getattr(lg, '_lddl_amd', False):
            h = logging.StreamHandler()
            h.setFormatter(logging.Formatter(_FMT))
            lg.addHandler(h)
            if self._log_dir is not None:
                fh = logging.FileHandler(os.path.join(self._log_dir, '{}.txt'.format(name)))
                fh.setFormatter(logging.Formatter(_FMT))
                lg.addHandler(fh)
            lg._lddl_amd = True
        lg.setLevel(self._log_level)
        return lg

    def init_for_worker(self, worker_rank):
        if self._worker_rank is None:
            self._worker_rank = worker_rank
            self._create(_name(self._node_rank, self._local_rank, worker_rank))

    def to(self, which):
        assert which in ('node', 'rank', 'worker')
        w0 = self._worker_rank is None or self._worker_rank == 0
        if which == 'node':
            return logging.getLogger(_name(self._node_rank)) if (
                self._local_rank == 0 and w0) else DummyLogger()
        if which == 'rank':
            return logging.getLogger(_name(self._node_rank, self._local_rank)) if w0 else \
                DummyLogger()
        return logging.getLogger(_name(self._node_rank, self._local_rank, self._worker_rank))
