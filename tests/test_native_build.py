"""The native libraries build for gfx950 and expose every symbol the bindings use (CPU-only check)."""
import ctypes

from cain_amd import ops
from cain_amd.energy import native


def test_kernel_library_loads_and_binds():
    lib = ops.load()
    for sym in ("cain_skinny_gemm_ex", "cain_gemm", "cain_gemm_ws_bytes", "cain_rmsnorm", "cain_embed", "cain_attention", "cain_sample",
                "cain_plan_create", "cain_plan_forward", "cain_plan_capture", "cain_graph_launch",
                "cain_graph_destroy", "cain_sample_params_size", "cain_rows_size", "cain_plan_desc_size"):
        assert hasattr(lib, sym), sym


def test_struct_layouts_match_native():
    from cain_amd.engine.engine import _CainLayer, _CainPlanDesc, _CainRows

    lib = ops.load()
    assert lib.cain_plan_desc_size() == ctypes.sizeof(_CainPlanDesc)
    assert lib.cain_rows_size() == ctypes.sizeof(_CainRows)
    assert lib.cain_layer_size() == ctypes.sizeof(_CainLayer)
    assert lib.cain_sample_params_size() == ops.SAMPLE_BYTES == 48


def test_energy_library_loads_without_gpu():
    lib = native.load()
    assert lib.es_sample_size() == ctypes.sizeof(native.ESample)
    assert native.init() >= 0


def test_default_kernel_library_links_no_vendor_gemm():
    """Every GEMM is a hand-written kernel: the library the engine and the headline load links no vendor GEMM
    library and has no library-GEMM hook (the round-3 hipBLASLt A/B path is gone)."""
    import subprocess

    lib = ops.load()
    assert not hasattr(lib, "cain_lt_gemm") and not hasattr(lib, "cain_set_lt_api")
    assert hasattr(lib, "cain_gemm_w4") and not hasattr(lib, "cain_front")
    needed = subprocess.run(["readelf", "-d", str(ops.LIB_PATH)], capture_output=True, text=True).stdout
    assert "hipblaslt" not in needed.lower() and "rocblas" not in needed.lower(), needed
