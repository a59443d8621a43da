import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, 'tests', 'golden')
ASSETS = os.path.join(REPO, 'lddl_amd', 'assets')
VOCAB_UNCASED = os.path.join(ASSETS, 'vocab_synth_uncased_30522.txt')
VOCAB_CASED = os.path.join(ASSETS, 'vocab_synth_cased_28996.txt')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (run with -m gpu)')
