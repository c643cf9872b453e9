"""Binary on-disk batches — the "CTRBIN01" format of csrc/io.cpp.

The reference parses its encoded CSV text (`label,idx_1..idx_F` per line, written by
``src/encode/data_.py:85``) on every run: ``pd.read_csv(...).values.astype(int)`` in
``all_main/pretrain_main.py:50-53``, ``islice`` + ``str.split`` per line in the RL drivers
(``hybrid_td3_main_per_v10.py:348-351``). Here the text is converted ONCE by the native
streaming parser (``ctr_csv_to_bin``) into a 64-byte header + an int32 ``[rows, 1+F]``
matrix that is memory-mapped afterwards: no parsing, no full-file copy, and whole batches
go host -> device as one contiguous slice.

    csv_to_bin("train_.txt", "train_.bin")        # once
    data = open_bin("train_.bin")                  # np.memmap int32 [N, 1+F]
    ds = libsvm_dataset(data[:, 1:], data[:, 0])   # unchanged reference dataset API
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

from ._lib import lib

HEADER_BYTES = 64


def csv_to_bin(csv_path: str | os.PathLike, bin_path: str | os.PathLike) -> tuple[int, int, int]:
    """Convert an encoded CSV file; returns (rows, cols, max feature id)."""
    rows, cols, max_id = C.c_int64(), C.c_int32(), C.c_int64()
    lib.ctr_csv_to_bin(os.fsencode(csv_path), os.fsencode(bin_path), C.byref(rows),
                       C.byref(cols), C.byref(max_id))
    return rows.value, cols.value, max_id.value


def bin_info(bin_path: str | os.PathLike) -> dict:
    rows, cols, max_id, off = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int64()
    lib.ctr_bin_info(os.fsencode(bin_path), C.byref(rows), C.byref(cols), C.byref(max_id),
                     C.byref(off))
    return {"rows": rows.value, "cols": cols.value, "max_id": max_id.value,
            "data_offset": off.value}


def open_bin(bin_path: str | os.PathLike) -> np.ndarray:
    """The file's int32 [rows, cols] matrix, memory-mapped read-only (validated header)."""
    info = bin_info(bin_path)
    if info["rows"] == 0:
        return np.zeros((0, info["cols"]), dtype=np.int32)
    return np.memmap(bin_path, dtype="<i4", mode="r", offset=info["data_offset"],
                     shape=(info["rows"], info["cols"]))


def load_encoded(csv_path: str | os.PathLike, cache: bool = True) -> np.ndarray:
    """The values ``pd.read_csv(csv_path, header=None).values.astype(int)`` gives, through a
    binary sidecar ``<csv>.ctrbin`` (built on first use, rebuilt when the CSV is newer)."""
    csv_path = Path(csv_path)
    bin_path = csv_path.with_name(csv_path.name + ".ctrbin")
    if not cache:
        bin_path = bin_path.with_name(bin_path.name + f".{os.getpid()}")
    if not bin_path.exists() or bin_path.stat().st_mtime < csv_path.stat().st_mtime:
        tmp = bin_path.with_name(bin_path.name + f".tmp{os.getpid()}")
        csv_to_bin(csv_path, tmp)
        os.replace(tmp, bin_path)
    data = open_bin(bin_path)
    if not cache:
        data = np.array(data)
        bin_path.unlink()
    return data
