"""lddl_amd — MI355X-native BERT preprocessing hot path of LDDL."""
__version__ = '0.1.0'
