"""Layout / format helpers with the reference's contracts (lddl/utils.py:33-109,
lddl/download/utils.py:42-51). The output layout is detected from file names only:
a file belongs to the dataset iff its extension contains '.parquet'; it is binned iff that
extension contains '_' and its bin id is the integer after the last '_'."""
import io
import os
import pathlib

import numpy as np
import pyarrow.parquet as pq


def mkdir(d):
    pathlib.Path(d).mkdir(parents=True, exist_ok=True)


def expand_outdir_and_mkdir(outdir):
    outdir = os.path.abspath(os.path.expanduser(outdir))
    mkdir(outdir)
    return outdir


def get_all_files_paths_under(root):
    for r, _, files in os.walk(root):
        for f in files:
            yield os.path.join(r, f)


def get_all_parquets_under(path):
    return sorted(p for p in get_all_files_paths_under(path)
                  if '.parquet' in os.path.splitext(p)[1])


def _ext(p):
    return os.path.splitext(p)[1]


def get_all_bin_ids(file_paths):
    ids = sorted({int(_ext(p).split('_')[-1]) for p in file_paths if '_' in _ext(p)})
    if ids != list(range(len(ids))):
        raise ValueError('bin id must be contiguous integers starting from 0!')
    return ids


def get_file_paths_for_bin_id(file_paths, bin_id):
    want = '.parquet_{}'.format(bin_id)
    return [p for p in file_paths if _ext(p) == want]


def get_num_samples_of_parquet(path):
    return pq.ParquetFile(path).metadata.num_rows


def attach_bool_arg(parser, flag_name, default=False, help_str=None):
    dest = flag_name.replace('-', '_')
    h = help_str if help_str is not None else flag_name.replace('-', ' ')
    parser.add_argument('--' + flag_name, dest=dest, action='store_true', help=h)
    parser.add_argument('--no-' + flag_name, dest=dest, action='store_false', help=h)
    parser.set_defaults(**{dest: default})


def serialize_np_array(a):
    buf = io.BytesIO()
    np.save(buf, a)
    return buf.getvalue()


def deserialize_np_array(b):
    return np.load(io.BytesIO(b))


def parse_str_of_num_bytes(s, return_str=False):
    """'<float>[kKmMgG]' -> bytes. Like the reference, the last character is always taken as
    the unit, so a bare number loses its last digit ('1024' -> 102)."""
    try:
        power = 'kmg'.find(s[-1].lower()) + 1
        size = float(s[:-1]) * 1024 ** power
    except ValueError:
        raise ValueError('Invalid size: {}'.format(s))
    return s if return_str else int(size)
