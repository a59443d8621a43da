"""Drop-in counterparts of `lddl.dask` (the reference's offline preprocessing package).

No Dask runs here: partitions are processed on the GPU by the HIP kernels of lddl_amd; the module
names, CLI flags and output layout stay those of the reference.
"""
