"""Console scripts with the reference's names (setup.py:63-74 of wdykas/LDDL); the native library
is built in-tree by `python -m lddl_amd.build` (hipcc --offload-arch=gfx950)."""
from setuptools import find_packages, setup

setup(
    name='lddl_amd',
    version='0.1.0',
    description='MI355X-native BERT preprocessing hot path of LDDL',
    packages=find_packages(include=['lddl_amd', 'lddl_amd.*']),
    package_data={'lddl_amd': ['assets/*', '_lib/*.so']},
    python_requires='>=3.8',
    install_requires=['numpy', 'pyarrow', 'torch'],
    entry_points={
        'console_scripts': [
            'preprocess_bert_pretrain=lddl_amd.dask.bert.pretrain:console_script',
            'balance_dask_output=lddl_amd.dask.load_balance:console_script',
            'generate_num_samples_cache=lddl_amd.dask.load_balance:generate_num_samples_cache',
        ],
    },
)
