"""The drop-in boundary: libsiddhi_hip.so loads on any host and exports every symbol that
include/siddhi_hip.h declares (no compute call is made without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "siddhi_hip.h")).read()
    return sorted(set(re.findall(r"\b(sdh_\w+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("sdh_engine_create", "sdh_engine_push", "sdh_engine_poll", "sdh_engine_flush",
              "sdh_engine_snapshot", "sdh_engine_restore", "sdh_engine_destroy", "sdh_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from siddhi_amd.engine import LIB_PATH, load_library
    assert os.path.exists(LIB_PATH), "build() must produce siddhi_amd/libsiddhi_hip.so"
    lib = load_library()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert b"gfx950" in lib.sdh_version()


def test_gfx950_code_object_present():
    data = open(os.path.join(ROOT, "siddhi_amd", "libsiddhi_hip.so"), "rb").read()
    assert b"gfx950" in data
