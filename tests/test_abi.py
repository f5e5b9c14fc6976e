"""The C-ABI library loads and exports every symbol include/*.h declares
(no device calls: this container has no GPU)."""
import ctypes
import os
import re

import gbgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gb(?:gpu)?_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol():
    lib = gbgpu.load()
    names = declared("gbgpu.h") + declared("gbgpu_synth.h")
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(gbgpu.EXPORTS)


def test_abi_version_and_errors():
    lib = gbgpu.load()
    assert lib.gbgpu_abi_version() == 13
    assert b"unsupported" in lib.gbgpu_strerror(gbgpu.GBGPU_EUNSUPPORTED) or \
        b"not supported" in lib.gbgpu_strerror(gbgpu.GBGPU_EUNSUPPORTED)


def test_open_fails_loudly_without_device():
    import torch
    if torch.cuda.device_count() > 0:
        return
    ctx = ctypes.c_void_p()
    rc = gbgpu.load().gbgpu_open(0, ctypes.byref(ctx))
    assert rc == gbgpu.GBGPU_ENODEVICE


def test_merge_topk_msg3a_semantics():
    # Msg3a::mergeLists: score desc, ties -> lower docid, duplicates dropped
    a = (np.array([5, 3, 9], np.int64), np.array([9.0, 7.0, 7.0], np.float32))
    b = (np.array([4, 1, 3], np.int64), np.array([8.0, 7.0, 7.0], np.float32))
    d, s = gbgpu.merge_topk([a, b], 5)
    assert d.tolist() == [5, 4, 1, 3, 9]
    assert s.tolist() == [9.0, 8.0, 7.0, 7.0, 7.0]


import numpy as np  # noqa: E402
