"""Drop-in counterparts of lddl.torch (the reference's PyTorch loader package).

`get_bert_pretrain_data_loader` is resolved lazily, so that DataLoader workers started with
`spawn` / `forkserver` import only the worker-side modules (`packing`, `datasets`), never the
native library."""


def __getattr__(name):
    if name == 'get_bert_pretrain_data_loader':
        from .bert import get_bert_pretrain_data_loader
        return get_bert_pretrain_data_loader
    raise AttributeError(name)
