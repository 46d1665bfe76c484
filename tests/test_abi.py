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


def _create(lib, blob, device=0):
    from siddhi_amd.engine import SdhConfig
    cfg = SdhConfig(device=device, shard_rank=0, shard_world=1)
    h = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(blob, max(1, len(blob)))
    rc = lib.sdh_engine_create(buf, len(blob), ctypes.byref(cfg), ctypes.byref(h))
    return rc, h


def test_malformed_program_is_invalid_without_a_device():
    """sdh_engine_create validates the program before any device call: a malformed blob fails with
    SDH_E_INVALID and sdh_last_error(NULL) says why (the reference's SiddhiAppCreationException)."""
    from siddhi_amd.engine import load_library
    lib = load_library()
    for blob, why in ((b"", b"magic"), (b"NOT-AN-IR-BLOB-AT-ALL", b"magic"),
                      (b"SDHIR001" + (7).to_bytes(8, "little"), b"version"),
                      (b"SDHIR001" + (2).to_bytes(8, "little") + (3).to_bytes(8, "little"), b"truncated")):
        rc, h = _create(lib, blob)
        assert rc == -1 and not h.value, (blob, rc)
        assert why in lib.sdh_last_error(None).lower(), lib.sdh_last_error(None)


def test_null_arguments_are_invalid():
    from siddhi_amd.engine import load_library
    lib = load_library()
    assert lib.sdh_engine_create(None, 0, None, None) == -1
    assert lib.sdh_engine_push(None, 0, None) == -1
    assert lib.sdh_engine_poll(None, None) == -1
    assert lib.sdh_engine_poll_device(None, None) == -1
    assert lib.sdh_engine_flush(None) == -1
    assert lib.sdh_engine_restore(None, None, 0) == -1
    lib.sdh_engine_destroy(None)  # no-op


def test_valid_program_needs_a_device():
    """A well-formed program on a host with no HIP device fails loudly (SDH_E_DEVICE): the engine has
    no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        import pytest
        pytest.skip("a device is present")
    from siddhi_amd import ql
    from siddhi_amd.engine import load_library
    from siddhi_amd.planner import plan
    from siddhi_amd.workloads import c1_app
    lib = load_library()
    rc, h = _create(lib, plan(ql.parse(c1_app())).serialize())
    assert rc == -3 and not h.value
    assert b"no hip device" in lib.sdh_last_error(None).lower()


def test_shape_compiled_kernels_build_without_a_device():
    """spec.hip's generated K_seq / K_part sources (register tables on and off) compile for gfx950
    through hiprtc on a host with no GPU."""
    from siddhi_amd.engine import load_library
    lib = load_library()
    lib.sdh_spec_selftest.restype = ctypes.c_int
    log = ctypes.create_string_buffer(8192)
    n = lib.sdh_spec_selftest(log, len(log))
    assert n == 7, log.value.decode(errors="replace")


def _c1_abi():
    """tests/native/c1_abi: the C host built from include/ alone (make builds it when missing)."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    exe = os.path.join(here, "native", "c1_abi")
    subprocess.check_call(["make", "-s", "-C", os.path.join(here, "native"), "c1_abi"])
    return exe


def test_c_host_builds_the_program_blob_from_the_header(tmp_path):
    """A C program that sees only include/siddhi_hip.h and include/siddhi_hip_ir.h builds the C1
    program blob by hand: byte for byte the blob the planner serializes for the same query."""
    import subprocess
    from siddhi_amd import ql
    from siddhi_amd.planner import plan
    from siddhi_amd.workloads import c1_app
    out = tmp_path / "c1.blob"
    subprocess.check_call([_c1_abi(), "blob", str(out)])
    assert out.read_bytes() == plan(ql.parse(c1_app())).serialize()


def test_ir_header_constants_match_the_planner():
    """include/siddhi_hip_ir.h's constants are the ones siddhi_amd/ir.py writes."""
    from siddhi_amd import ir
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                             "siddhi_hip_ir.h")).read()
    defs = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"#define SDH_(\w+) \(?(-?\d+)\)?", text))
    for name in ("T_INT", "T_LONG", "T_FLOAT", "T_DOUBLE", "T_BOOL", "T_STRING", "OP_CONST", "OP_ATTR",
                 "OP_IS_NULL", "OP_STREAM_IS_NULL", "OP_CMP", "OP_AND", "OP_OR", "OP_NOT", "OP_ARITH", "CMP_EQ",
                 "CMP_NE", "CMP_GT", "CMP_GE", "CMP_LT", "CMP_LE", "AR_ADD", "AR_SUB", "AR_MUL", "AR_DIV", "AR_MOD",
                 "IDX_CURRENT", "IDX_LAST", "K_STREAM", "K_COUNT", "K_LOGICAL", "K_ABSENT", "L_AND", "L_OR",
                 "Q_PATTERN", "Q_SEQUENCE", "R_SINGLE", "R_MULTI", "N_STREAM", "N_NEXT", "N_EVERY", "N_LOGICAL",
                 "N_COUNT"):
        assert defs[name] == getattr(ir, name), name
    assert defs["IR_VERSION"] == ir.VERSION
    assert f'"{ir.MAGIC.decode()}"' in text
