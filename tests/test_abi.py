"""The C-ABI boundary (include/aquad.h) without a GPU: the library builds, loads, exports every
declared symbol, and the host-side observable surface matches the reference's."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "aquad.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(aq_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from ppls_amd import _lib
    return _lib.load()


def test_header_declares_expected_api():
    fns = header_functions()
    from ppls_amd import _lib
    assert fns == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (aq_[a-z0-9_]+)$", out, flags=re.M))
    assert set(header_functions()) <= exported


def test_library_is_gfx950_code_object(lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", lib._name], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(lib._name, "rb").read()
    assert b"gfx950" in blob


def test_strerror_and_arg_validation(lib):
    import ctypes
    assert lib.aq_strerror(0) == b"ok"
    assert lib.aq_strerror(-5) == b"maximum refinement depth reached"
    assert lib.aq_strerror(-9) == b"the persistent grid cannot be co-resident on the device"
    # NULL context / arguments are rejected before any device call
    assert lib.aq_integrate(None, None, None) == -1
    assert lib.aq_fetch(None, 0, None) == -1
    assert lib.aq_level_step(None, 0, None, 0, None, 0, 1e-3, 0, 64, None, None) == -1
    assert lib.aq_level_step_chained(None, 0, None, None, 0, None, 0, 1e-3, 0, 64, None, None) == -1
    n = ctypes.c_int(-1)
    rc = lib.aq_device_count(ctypes.byref(n))
    assert (rc == 0) == (n.value > 0)


def test_cli_numprocs_error_matches_reference():
    """aquadPartA.c:86-90: numprocs < 2 -> that exact stderr line and exit(1)."""
    from ppls_amd import build
    build.build()
    p = subprocess.run([build.CLI, "-n", "1"], capture_output=True, text=True)
    assert p.returncode == 1
    assert p.stderr == "ERROR: Must have at least 2 processes to run\n"
    assert p.stdout == ""


def test_python_farmer_numprocs_error():
    from ppls_amd import AquadError, farmer
    with pytest.raises(AquadError, match="ERROR: Must have at least 2 processes to run"):
        farmer(1)


@pytest.mark.parametrize("name", ["cosh4_eps1e-3", "cosh4_eps1e-10", "sin_recip_eps1e-9"])
def test_format_reference_is_byte_identical(trees, name):
    """main()'s printout (aquadPartA.c:107-117) for the reference's own numbers."""
    from ppls_amd import format_reference
    ref = trees[name]["reference"]
    area = float(ref["area_printed"])
    assert format_reference(area, ref["tasks_per_process"]) == ref["stdout"]


def test_group_tasks_deals_cus_round_robin():
    from ppls_amd.aquad import group_tasks
    assert group_tasks({5: 1, 1: 10, 9: 100}, 2) == [10 + 100, 1]
    assert sum(group_tasks({i: i for i in range(256)}, 4)) == sum(range(256))


def test_print_reference_from_result(lib, tmp_path, trees):
    """aq_print_reference(FILE*, const aq_result*) -- main()'s printout (aquadPartA.c:107-117) from a
    result struct: farmer 0, then one column per GPU (tasks_per_gpu)."""
    import ctypes
    import numpy as np
    from ppls_amd import _lib, format_reference
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    per_gpu = np.array([1679, 1605, 1682, 1601], np.uint64)   # the header's sample split (:34-36)
    r = _lib.aq_result()
    r.area = 7583461.801486495
    r.tasks = int(per_gpu.sum())
    r.n_gpus = 4
    r.tasks_per_gpu = per_gpu.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
    path = tmp_path / "out.txt"
    f = libc.fopen(str(path).encode(), b"w")
    lib.aq_print_reference(f, ctypes.byref(r))
    lib.aq_print_reference_procs(f, 7583461.801486495, (ctypes.c_uint64 * 2)(0, 6567), 2)
    libc.fclose(f)
    text = path.read_text()
    want = format_reference(r.area, [0] + [int(v) for v in per_gpu])
    assert text.startswith(want)
    assert text[len(want):] == format_reference(r.area, [0, 6567])
    assert want.splitlines()[0] == "Area=7583461.801486"


def test_exact_round_is_exported_host_code(lib):
    """aq_exact_round runs on the host (no GPU): limbs of 1.5 * 2^0 round to 1.5."""
    import ctypes
    import numpy as np
    limbs = np.zeros(68, np.int64)
    # 1.5 = 3 * 2^-1 -> bit position -1 + 1088 = 1087 -> limb 33, bit 31
    limbs[33] = 3 << 31 & 0xffffffff
    limbs[34] = (3 << 31) >> 32
    assert lib.aq_exact_round(limbs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))) == 1.5


def test_user_integrand_name(lib):
    assert lib.aq_user_integrand_name().startswith(b"gauss")


@pytest.mark.skipif(not os.path.exists("/opt/conda/include/mpi.h"), reason="no MPI headers in this image")
def test_integration_mpi_binding_compiles(tmp_path):
    """INTEGRATION.md §1's C + MPI binding compiles (warnings as errors) against include/aquad.h, so
    the documented boundary cannot drift from the header."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    src = re.search(r"```c\n(.*?)```", doc, re.S).group(1)
    c = tmp_path / "aquadPartA_gpu.c"
    c.write_text(src)
    subprocess.run(["gcc", "-Wall", "-Wextra", "-Werror", "-c", "-I/opt/conda/include", "-I", os.path.join(ROOT, "include"),
                    "-o", str(tmp_path / "b.o"), str(c)], check=True, capture_output=True, text=True, timeout=60)


def test_oracle_seed_depth_rule_matches_library(lib):
    """The oracle partition's seed depth (tests' device_seed_S: floor(log2 V) + S) equals the
    library's own (aq_seed_depth = aq_stream.h seed_depth_job) for every V a launch can have."""
    import ctypes
    from conftest import device_seed_S
    f = lib.aq_seed_depth
    f.argtypes = [ctypes.c_ulonglong]
    f.restype = ctypes.c_int
    for V in list(range(1, 4097)) + [6144, 9216, 15360, 24576, 3072 * 16]:
        assert f(V) == (V.bit_length() - 1) + device_seed_S(V, 1), V
