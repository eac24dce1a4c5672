"""CPU-only checks of the C-ABI boundary: the HIP library loads, exports every function that
include/vss.h declares, and validates arguments without touching a GPU."""
import ctypes
import os
import re

import pytest

from vss_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(N.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int64_t|int|const char\*)\s+(vss_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_expected_entry_points():
    assert declared_functions() == sorted(N.EXPORTED)


def test_library_loads_and_exports_every_declared_symbol():
    if not os.path.exists(N.LIB_PATH):
        from vss_amd import build
        build()
    lib = N.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.vss_abi_version() == N.ABI_VERSION


def test_library_is_built_from_the_tree_sources():
    """The library's source stamp equals the hash of the sources in this tree, and a library whose
    stamp differs (a stale prebuilt .so that travelled with the tree) is refused."""
    lib = N.load()
    N.verify_source_hash(lib)
    with pytest.raises(N.NativeError, match="built from other sources"):
        N.verify_source_hash(lib, expected="0" * 16)


def test_library_without_stamp_symbol_is_refused():
    """A library older than the stamp (no vss_source_hash symbol) raises NativeError with the rebuild
    hint, not an AttributeError."""
    class NoStamp:  # ctypes.CDLL raises AttributeError for a symbol the library does not export
        def __getattr__(self, name):
            raise AttributeError(name)
    with pytest.raises(N.NativeError, match="make -C"):
        N.verify_source_hash(NoStamp())


def test_stale_library_is_refused_at_load(tmp_path, monkeypatch):
    """load() itself refuses a library whose stamp does not match the tree (here: the tree's
    stamped sources replaced by a modified copy of one of them)."""
    import shutil
    src = os.path.join(tmp_path, "vss_step.hip")
    shutil.copy(N.STAMPED[0], src)
    with open(src, "a") as f:
        f.write("// edited after the build\n")
    monkeypatch.setattr(N, "STAMPED", (src,) + tuple(N.STAMPED[1:]))
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(N.NativeError, match="built from other sources"):
        N.load()


def test_error_strings():
    lib = N.load()
    assert lib.vss_error_string(0) == b"ok"
    assert b"invalid" in lib.vss_error_string(1)
    assert b"launch" in lib.vss_error_string(2)


def test_argument_validation_without_gpu():
    """Calls with null/invalid arguments are rejected before any HIP call is made."""
    lib = N.load()
    prm = N.VssParams(10, 2, 3, 0, 1, 400, 1)
    st = N.VssState()  # all null
    io = N.VssStepIO()
    assert lib.vss_step(None, 16, 0, ctypes.byref(prm), ctypes.byref(st), ctypes.byref(io)) == 1
    assert lib.vss_step(None, -1, 0, ctypes.byref(prm), None, None) == 1
    assert lib.vss_reset_dones(None, 16, ctypes.byref(prm), ctypes.byref(st)) == 1
    assert lib.vss_compute_observations(None, 16, ctypes.byref(st), None, 6) == 1
    fake = ctypes.c_void_p(16)  # never dereferenced: rejected on n_agents / mode first
    st2 = N.VssState(fake, fake, fake, fake, fake)
    assert lib.vss_compute_observations(None, 16, ctypes.byref(st2), fake, 5) == 1
    assert lib.vss_step(None, 16, 7, ctypes.byref(prm), ctypes.byref(st2), ctypes.byref(io)) == 1


def test_struct_layouts_match_header():
    """ctypes mirrors of vss_params / vss_state / vss_step_io have the C layout."""
    assert ctypes.sizeof(N.VssParams) == 32
    assert N.VssParams.seed.offset == 24
    assert ctypes.sizeof(N.VssState) == 5 * 8
    assert ctypes.sizeof(N.VssStepIO) == 9 * 8


def test_product_path_refuses_cpu():
    from envs.vss import VSS, default_cfg
    with pytest.raises(N.NativeError):
        VSS(default_cfg(16), "cpu", "cpu", 0, True, False, False)


def test_oracle_under_asan_ubsan():
    """The CPU restatement driven through every mode / size under ASan + UBSan (host sanitizers;
    GPU sanitizers are not available on the MI355X pool)."""
    import subprocess
    r = subprocess.run(["make", "-s", "-C", os.path.join(os.path.dirname(N.HEADER), "..", "oracle"), "check-asan"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "oracle selftest ok" in r.stdout


def test_c_host_demo_compiles_and_links(tmp_path):
    """examples/vss_host_demo.c — the C ABI from plain C (hipMalloc'd buffers, no Python) —
    compiles against include/vss.h and links against the built library (run: tests/test_c_host.py)."""
    import shutil
    import subprocess
    if not shutil.which("gcc") or not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("gcc or the HIP headers are not available")
    if not os.path.exists(N.LIB_PATH):
        from vss_amd import build
        build()
    out = os.path.join(tmp_path, "vss_host_demo")
    r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "examples"), f"OUT={out}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(out)
