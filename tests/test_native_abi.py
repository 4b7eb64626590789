"""The C-ABI boundary without a GPU: libraries load, export exactly what include/*.h declares,
and reject bad arguments with an error code + message (never exit(), unlike the reference's
gpuErrchk, generateCUDACode.py:106-112). No compute call is made here."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

from biped_pympc_amd import _native, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", src, flags=re.M):
            if m.group(1) not in ("if", "defined"):
                names.add(m.group(1))
    return names


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True)
    return {line.split()[-1] for line in out.stdout.splitlines() if " T " in line}


def test_header_declares_the_cusadi_symbol_and_extended_api():
    names = _declared_functions()
    assert "evaluate" in names
    assert {"srbd_qp_former", "srbd_pdipm", "srbd_pdipm_cold", "srbd_pdipm_ccs", "srbd_mpc_solve",
            "srbd_mpc_solve_fused", "srbd_mpc_step", "srbd_last_error", "srbd_abi_version"} <= names


def test_core_library_exports_every_declared_symbol():
    build.build()
    exports = _exports(_native.lib_path())
    missing = (_declared_functions() - {"evaluate"}) - exports
    assert not missing, missing


@pytest.mark.parametrize("fn,N,K", build.DROPIN_CONFIGS)
def test_dropin_libraries_export_evaluate(fn, N, K):
    path = os.path.join(build.LIB_DIR, build.dropin_lib_name(fn, N, K))
    assert os.path.exists(path)
    assert "evaluate" in _exports(path)
    lib = ctypes.CDLL(path)  # resolves libsrbd_mpc.so through rpath $ORIGIN
    assert lib.evaluate


def test_reference_library_names():
    # CusadiFunction loads lib{fn.name()}.so (CusadiFunction.py:30; setup.sh:10-11)
    assert build.dropin_lib_name("qp_former", 10, None) == "libqp_former.so"
    assert build.dropin_lib_name("sparse_pdipm_multiple_iterations", 10, 5) == \
        "libsparse_pdipm_multiple_iterations.so"


def test_abi_introspection():
    L = _native.lib()
    assert L.srbd_abi_version() == 1
    for N in (1, 10, 20, 32):
        lds = L.srbd_solver_lds_bytes(N)
        assert 0 < lds <= 160 * 1024
    assert L.srbd_solver_lds_bytes(0) == 0 and L.srbd_solver_lds_bytes(33) == 0
    assert L.srbd_mpc_workspace_doubles(10, 4096) == 4096 * 2256
    # one fallback scratch slot: the general solve's working set at its largest horizon (host-only);
    # 2048 of them (+ lock words) are the per-device pool INTEGRATION.md prices at 332 MB
    assert L.srbd_scratch_slot_bytes() == 162000
    assert L.srbd_set_scratch_slots(-1) != 0 and "slots >= 0" in _native.last_error()


def test_bad_arguments_return_errors_without_touching_the_gpu():
    L = _native.lib()
    nulls = _native.ptr_array([0] * 17)
    assert L.srbd_qp_former(0, 4, nulls, nulls, None) != 0
    assert "bad arguments" in _native.last_error()
    assert L.srbd_pdipm(10, 0, 4, nulls, nulls, None) != 0  # n_iter must be >= 1
    assert L.srbd_pdipm(10, 5, 4, nulls, nulls, None) != 0  # null pointers
    assert "null input" in _native.last_error()
    assert L.srbd_evaluate_pdipm(40, 5, None, None, None, 4) < 0
    # an empty batch is a successful no-op, whatever the (zero-size) buffers point to
    assert L.srbd_qp_former(10, 0, nulls, nulls, None) == 0
    assert L.srbd_pdipm(10, 5, 0, nulls, nulls, None) == 0
    assert L.srbd_pdipm_cold(10, 5, 0, 1.0, nulls, nulls, None) == 0
    assert L.srbd_pdipm_ccs(10, 5, 4, nulls, nulls, None) != 0
    assert "x_init" in _native.last_error()
    # the one-launch controller step: any horizon 1..32, prep required
    prep = _native.MPCPrep()
    assert L.srbd_mpc_step(40, 20, 4, 1.0, ctypes.byref(prep), None, None, None, 0, None, None, None, None) != 0
    assert "bad horizon" in _native.last_error()
    assert L.srbd_mpc_step(15, 20, 4, 1.0, ctypes.byref(prep), None, None, None, 0, None, None, None, None) != 0
    assert "null foot_wrench" in _native.last_error()
    assert L.srbd_mpc_step(10, 20, 4, 1.0, None, None, None, None, 0, None, None, None, None) != 0
    assert L.srbd_mpc_step(10, 20, 4, 1.0, ctypes.byref(prep), None, None, None, 0, None, None, None, None) != 0
    assert L.srbd_mpc_step(10, 20, 0, 1.0, ctypes.byref(prep), None, None, None, 0, None, None, None, None) == 0


def test_build_id_is_the_source_hash():
    """Build provenance: libsrbd_mpc.so carries the hash of the sources and flags it was compiled
    from (build.py source_hash), readable both from the file and through srbd_build_id(); the drop-in
    shims carry the id of their own configuration over that core."""
    build.build()
    core = _native.lib_path()
    h = build.source_hash()
    assert build.embedded_id(core) == h
    L = ctypes.CDLL(core)
    L.srbd_build_id.restype = ctypes.c_char_p
    assert L.srbd_build_id().decode() == h
    for fn, N, K in build.DROPIN_CONFIGS:
        path = os.path.join(build.LIB_DIR, build.dropin_lib_name(fn, N, K))
        assert build.embedded_id(path) == build._shim_hash(fn, N, K, h)


def test_source_hash_tracks_content_not_mtime(tmp_path):
    """A touched source keeps the id; one edited byte changes it (build() rebuilds on a mismatch)."""
    srcs = build.core_sources()
    copy = tmp_path / os.path.basename(srcs[-1])
    copy.write_bytes(open(srcs[-1], "rb").read())
    h0 = build.source_hash(srcs[:-1] + [str(copy)])
    os.utime(copy, (1, 1))
    assert build.source_hash(srcs[:-1] + [str(copy)]) == h0
    copy.write_bytes(copy.read_bytes() + b" ")
    assert build.source_hash(srcs[:-1] + [str(copy)]) != h0
