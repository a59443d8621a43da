"""Drop-in counterparts of lddl.torch (the reference's PyTorch loader package)."""
