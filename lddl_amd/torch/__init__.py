"""Drop-in counterparts of lddl.torch (the reference's PyTorch loader package)."""
from .bert import get_bert_pretrain_data_loader  # noqa: F401
