"""lddl_utf8_check (csrc/utf8.hip) against Python's strict UTF-8 decoder: the first offset the
decoder rejects (UnicodeDecodeError.start), on valid text, every malformed-sequence class and a
seeded fuzz; and the CLI raising on malformed input as dask's read_text does."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _py_first_bad(b):
    try:
        b.decode('utf-8')
        return -1
    except UnicodeDecodeError as e:
        return e.start


def _gpu_first_bad(b):
    from lddl_amd.punkt import utf8_first_invalid
    t = torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda() if b else torch.zeros(
        0, dtype=torch.uint8, device='cuda')
    return utf8_first_invalid(t)


CASES = [b'', b'plain ascii', 'naïve café 漢字 \U0001F600 　'.encode(),
         b'\x80', b'a\xbf', b'\xc0\x80', b'\xc1\xbf', b'\xc2', b'\xc2\x41', b'\xe0\x80\x80',
         b'\xe0\x9f\xbf', b'\xed\xa0\x80', b'\xed\x9f\xbf', b'\xef\xbf', b'\xf0\x8f\xbf\xbf',
         b'\xf4\x90\x80\x80', b'\xf5\x80\x80\x80', b'\xff', b'abc\xe2\x82', b'\xe2\x82\xac\x80',
         b'\xf0\x9f\x98\x80\x80\x80\x80\x80', b'x' * 15 + b'\xe2\x82\xac' + b'y' * 30 + b'\x9f']


@pytest.mark.parametrize('i', range(len(CASES)))
def test_utf8_cases(i):
    b = CASES[i]
    assert _gpu_first_bad(b) == _py_first_bad(b)


def test_utf8_fuzz():
    rng = np.random.default_rng(7)
    good = 'the quick éè 中文 \U0001F680 brown'.encode()
    for _ in range(300):
        parts = []
        for _ in range(rng.integers(1, 40)):
            r = rng.random()
            if r < 0.7:
                parts.append(good[:rng.integers(0, len(good))])
            else:
                parts.append(bytes(rng.integers(0x7e, 0x100, rng.integers(1, 5)).astype(np.uint8)))
        b = b''.join(parts)
        assert _gpu_first_bad(b) == _py_first_bad(b), b


def test_cli_rejects_malformed_utf8(tmp_path):
    from conftest import VOCAB_UNCASED
    from lddl_amd.dask.bert import pretrain as P
    src = tmp_path / 'source' / 'en'
    src.mkdir(parents=True)
    (src / 'w.txt').write_bytes(b'wiki-1 good text here.\nwiki-2 bad \xff byte.\n')
    args = P.attach_args().parse_args(['--schedule', 'local', '--wikipedia', str(tmp_path / 'source'),
                                       '--sink', str(tmp_path / 'out'), '--vocab-file',
                                       VOCAB_UNCASED, '--sample-ratio', '1.0'])
    with pytest.raises(UnicodeDecodeError):
        P.main(args)
