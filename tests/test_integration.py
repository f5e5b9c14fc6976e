"""INTEGRATION.md's reference-side adapter compiles against the reference headers.

Every ```cpp block of INTEGRATION.md is concatenated, in order, after the
reference headers the adapter's host files include (Posdb.cpp:1-11,
Msg39.cpp, RdbList.cpp, Msg3a.cpp) and compiled with the reference's own flags
(Makefile:101: gnu++98, -fpermissive, -DPTHREADS), syntax only.  Needs the
reference tree, so it runs in the build container only (skipped elsewhere).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

PRELUDE = """\
#include "gb-include.h"
#include "Posdb.h"
#include "Query.h"
#include "Msg2.h"
#include "Msg39.h"
#include "TopTree.h"
#include "RdbList.h"
#include "Msg3a.h"
#include "Conf.h"
"""


def adapter_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```cpp\n(.*?)```", text, flags=re.S)
    assert len(blocks) >= 5, "INTEGRATION.md lost an adapter block"
    return PRELUDE + "\n".join(blocks)


def test_adapter_blocks_present():
    src = adapter_source()
    for fn in ("gbgpuIntersectLists", "gbgpuDocIdSplits", "gbgpuShardQuery", "gbgpuMergePosdb"):
        assert fn in src


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("g++") is None,
                    reason="reference tree or g++ absent (GPU box)")
def test_adapter_compiles_against_reference_headers(tmp_path):
    f = tmp_path / "gbgpu_adapter.cpp"
    f.write_text(adapter_source())
    cmd = ["g++", "-fsyntax-only", "-std=gnu++98", "-fpermissive", "-w", "-DPTHREADS",
           "-I" + REF, "-I" + os.path.join(ROOT, "include"), str(f)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("g++") is None,
                    reason="reference tree or g++ absent (GPU box)")
def test_adapter_has_no_null_path_at_O2(tmp_path):
    """Compiled as the reference builds (-O2), no path of the adapter may be a
    known null dereference: the reference's Mem.h turns malloc/calloc/realloc
    into a crash (Mem.h:221-225), which g++ then isolates into a trap -- the
    adapter must allocate with mmalloc/mfree as the reference's code does."""
    f = tmp_path / "gbgpu_adapter.cpp"
    f.write_text(adapter_source())
    cmd = ["g++", "-O2", "-c", "-std=gnu++98", "-fpermissive", "-w", "-Wnull-dereference", "-DPTHREADS",
           "-I" + REF, "-I" + os.path.join(ROOT, "include"), str(f), "-o", str(tmp_path / "a.o")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "null pointer dereference" not in r.stderr, r.stderr[-4000:]
