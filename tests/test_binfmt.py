"""CPU tests of the binary on-disk batch format (csrc/io.cpp, rl_ctr_prediction_amd.binfmt;
SURVEY.md §8f rank 2): the converted matrix is exactly what the reference's
``pd.read_csv(path, header=None).values.astype(int)`` reads (all_main/pretrain_main.py:50-53),
on the C1 toy files and on edge cases. Host code only: runs without a GPU."""
from __future__ import annotations

import os
import time

import numpy as np
import pandas as pd
import pytest

from conftest import ROOT

TOY = ROOT / "tests" / "golden" / "toy"


@pytest.fixture(scope="module")
def B():
    from rl_ctr_prediction_amd.build_lib import build
    try:
        build()
    except RuntimeError as e:  # no hipcc in this environment
        pytest.skip(str(e))
    from rl_ctr_prediction_amd import binfmt
    return binfmt


@pytest.mark.parametrize("name", ["train_.txt", "test_.txt"])
def test_toy_files_equal_pandas(B, tmp_path, name):
    ref = pd.read_csv(TOY / name, header=None).values.astype(int)
    rows, cols, max_id = B.csv_to_bin(TOY / name, tmp_path / "x.bin")
    assert (rows, cols) == ref.shape and max_id == ref[:, 1:].max()
    got = B.open_bin(tmp_path / "x.bin")
    assert got.dtype == np.int32
    np.testing.assert_array_equal(got, ref)


def _write(p, text):
    p.write_bytes(text.encode())
    return p


def test_line_endings_blank_lines_and_signs(B, tmp_path):
    csv = _write(tmp_path / "a.txt", "1,2,3\r\n0, 5 ,-7\n\n1,2147483647,0")  # no final newline
    B.csv_to_bin(csv, tmp_path / "a.bin")
    np.testing.assert_array_equal(B.open_bin(tmp_path / "a.bin"),
                                  [[1, 2, 3], [0, 5, -7], [1, 2147483647, 0]])
    assert B.bin_info(tmp_path / "a.bin")["max_id"] == 2147483647


def test_empty_file(B, tmp_path):
    B.csv_to_bin(_write(tmp_path / "e.txt", ""), tmp_path / "e.bin")
    assert B.open_bin(tmp_path / "e.bin").shape == (0, 0)


@pytest.mark.parametrize("text,match", [("1,2,3\n0,4\n", "line 2: 2 columns, expected 3"),
                                        ("1,2,x\n", "line 1: unexpected character"),
                                        ("1,,3\n", "line 1: empty or bad field"),
                                        ("1,2147483648\n", "line 1: bad integer"),
                                        ("1,2.5\n", "line 1: unexpected character")])
def test_malformed_input_fails_with_line(B, tmp_path, text, match):
    from rl_ctr_prediction_amd._lib import CtrHipError
    with pytest.raises(CtrHipError, match=match):
        B.csv_to_bin(_write(tmp_path / "m.txt", text), tmp_path / "m.bin")


def test_truncated_or_foreign_file_is_refused(B, tmp_path):
    from rl_ctr_prediction_amd._lib import CtrHipError
    B.csv_to_bin(TOY / "test_.txt", tmp_path / "t.bin")
    data = (tmp_path / "t.bin").read_bytes()
    (tmp_path / "cut.bin").write_bytes(data[:-4])
    with pytest.raises(CtrHipError, match="does not match"):
        B.open_bin(tmp_path / "cut.bin")
    (tmp_path / "bad.bin").write_bytes(b"NOTCTRBN" + data[8:])
    with pytest.raises(CtrHipError, match="not a CTRBIN01"):
        B.open_bin(tmp_path / "bad.bin")


def test_sidecar_cache_and_staleness(B, tmp_path):
    csv = _write(tmp_path / "train_.txt", "1,2,3\n0,4,5\n")
    a = B.load_encoded(csv)
    side = tmp_path / "train_.txt.ctrbin"
    assert side.exists()
    np.testing.assert_array_equal(a, [[1, 2, 3], [0, 4, 5]])
    time.sleep(0.01)
    _write(csv, "0,9,9\n")
    os.utime(csv, (side.stat().st_mtime + 5, side.stat().st_mtime + 5))
    np.testing.assert_array_equal(B.load_encoded(csv), [[0, 9, 9]])


def test_large_file_streams(B, tmp_path):
    """More rows than one 16 MiB read block and one write buffer: block boundaries split
    numbers and lines; the result still equals numpy's parse."""
    rng = np.random.default_rng(0)
    ref = np.concatenate([rng.integers(0, 2, (300_000, 1)), rng.integers(0, 10**9, (300_000, 22))],
                         axis=1)
    csv = tmp_path / "big.txt"
    np.savetxt(csv, ref, fmt="%d", delimiter=",")
    rows, cols, _ = B.csv_to_bin(csv, tmp_path / "big.bin")
    assert (rows, cols) == ref.shape
    np.testing.assert_array_equal(B.open_bin(tmp_path / "big.bin"), ref)
