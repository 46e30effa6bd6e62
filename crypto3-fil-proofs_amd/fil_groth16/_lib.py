"""Loads libfilgpu.so (the HIP kernels + C ABI of include/mi355x_groth16.h).

There is no CPU fallback: if the library is missing or no GPU is present, the compute entry points
raise.  Loading the library itself needs no GPU (symbols can be inspected on CPU-only hosts).
"""
import ctypes
import os

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("FILGPU_LIB", os.path.join(_PKG_ROOT, "build", "libfilgpu.so"))

# Every symbol declared in include/mi355x_groth16.h (checked by tests/test_abi.py)
EXPORTS = [
    "mi_device_count", "mi_ctx_create", "mi_ctx_destroy", "mi_last_error", "mi_ctx_stream", "mi_ctx_synchronize",
    "mi_ctx_set_caller_stream",
    "mi_circuit_load", "mi_circuit_info", "mi_circuit_free",
    "mi_srs_load", "mi_srs_generate", "mi_srs_export_vk", "mi_srs_export_query", "mi_srs_info", "mi_srs_free",
    "mi_groth16_prove", "mi_groth16_prove_dev", "mi_groth16_prove_batch", "mi_groth16_trapdoor_dlogs",
    "mi_msm_g1", "mi_msm_g2", "mi_ntt_fr",
    "mi_points_upload_g1", "mi_points_upload_g2", "mi_points_from_srs", "mi_points_free", "mi_points_count",
    "mi_msm_g1_dev", "mi_msm_g2_dev", "mi_ntt_fr_dev",
    "mi_ctx_get_stats", "mi_ctx_reset_stats", "mi_ctx_get_work", "mi_ctx_get_fallbacks", "mi_msm_window_bits",
    "mi_synth_generate", "mi_synth_generate_ex", "mi_synth_r1cs", "mi_synth_witness", "mi_synth_free",
    "mi_params_inspect", "mi_params_load", "mi_params_write", "mi_vk_write",
    "mi_groth16_verify", "mi_groth16_verify_batch", "mi_pairing",
    "mi_groth16_prove_share", "mi_groth16_prove_share_dev", "mi_groth16_assemble",
    "mi_groth16_prove_share_ranges", "mi_groth16_prove_share_ranges_dev",
    "mi_host_alloc", "mi_host_free", "mi_groth16_verify_batch_seeded",
    "mi_poseidon_constants", "mi_poseidon_hash", "mi_poseidon_hash_dev", "mi_tree_cache_size",
    "mi_tree_build", "mi_tree_build_dev", "mi_tree_c_build", "mi_tree_c_build_dev",
    "mi_tree_r_last_build", "mi_tree_r_last_build_dev",
    "mi_sdr_labels", "mi_sdr_labels_dev", "mi_sdr_labeling_proofs_dev", "mi_tree_inclusion_paths_dev", "mi_tree_d_inclusion_paths_dev",
    "mi_tree_d_build_dev", "mi_srs_msm_info", "mi_srs_table_state", "mi_srs_readmit", "mi_ctx_inject_oom",
    "mi_param_cache_id", "mi_param_cache_path", "mi_param_cache_metadata", "mi_get_groth_params",
    "mi_groth16_h_coeffs_dev", "mi_groth16_prove_share_ranges_h_dev", "mi_points_check_subgroup", "mi_points_info",
    "mi_groth16_prove_random", "mi_groth16_prove_dev_random", "mi_groth16_prove_batch_random",
    "mi_srs_stream_begin", "mi_srs_stream_part", "mi_srs_stream_end", "mi_srs_stream_abort", "mi_srs_export_query_dev",
    "mi_stacked_build", "mi_post_build", "mi_stacked_info", "mi_stacked_r1cs", "mi_stacked_load", "mi_stacked_public_inputs", "mi_stacked_witness_dev",
    "mi_stacked_witness", "mi_stacked_free", "mi_circuit_check_dev",
    "mi_points_precompute", "mi_points_table_info", "mi_ctx_get_table_msms", "mi_srs_window_tables",
    "mi_tune_set", "mi_tune_clear", "mi_tune_get", "mi_fq_check_read", "mi_srs_shared_la", "mi_ctx_get_shared_plans",
    "mi_ctx_get_derived_plans",
]

_lib = None


class FilGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libfilgpu error {code}: {msg}")
        self.code = code


def torch_sync(ctx):
    """Before a device-pointer entry: name torch's current stream on ctx's device as the library's caller stream
    (mi_ctx_set_caller_stream).  The C ABI then orders its first device access after the work queued there --
    the fill or copy that produced an input tensor, or an earlier reader of an output buffer -- with an event
    waited for on the device, not a host synchronisation (include/mi355x_groth16.h, "device pointers").  The
    entries return with their outputs written.  No-op without torch or before CUDA is initialised (the library's
    default caller stream, the legacy NULL stream, then covers every blocking stream).  The caller stream is a
    property of the context, so a Context is meant to be driven from one Python thread (as the C ABI's threading
    rule says); two threads on one context with different torch streams would race between this call and the
    entry that follows it."""
    import sys

    t = sys.modules.get("torch")
    if t is not None and t.cuda.is_initialized():
        dev = getattr(ctx, "device", 0)
        if "mi_ctx_set_caller_stream" in lib().missing_symbols:  # a pre-round-5 library: host synchronisation
            t.cuda.current_stream(dev).synchronize()
            return
        check(lib().mi_ctx_set_caller_stream(ctx.h, ctypes.c_void_p(t.cuda.current_stream(dev).cuda_stream or None)))


def build():
    import subprocess

    subprocess.check_call(["make", "-s", "-C", _PKG_ROOT, "-j8"])


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(
            f"{LIB_PATH} not found: build it with `make -C {_PKG_ROOT}` (HIP extension is required; "
            "there is no CPU fallback)")
    # One HIP runtime per process: torch's libtorch_hip NEEDs "libamdhip64.so" while this library
    # NEEDs "libamdhip64.so.7".  Loading torch first makes our dependency resolve to the runtime
    # torch already mapped (same SONAME); the other order maps two HIP/HSA runtimes into one process
    # and torch then reports "No HIP GPUs are available".
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, u8p, u64, c_int = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "mi_device_count": ([ctypes.POINTER(c_int)], c_int),
        "mi_ctx_create": ([c_int, pp], c_int),
        "mi_ctx_destroy": ([vp], None),
        "mi_last_error": ([], ctypes.c_char_p),
        "mi_ctx_stream": ([vp, pp], c_int),
        "mi_ctx_synchronize": ([vp], c_int),
        "mi_ctx_set_caller_stream": ([vp, vp], c_int),
        "mi_circuit_load": ([vp, vp, pp], c_int),
        "mi_circuit_info": ([vp, vp], c_int),
        "mi_circuit_free": ([vp], None),
        "mi_srs_load": ([vp, vp, vp, c_int, pp], c_int),
        "mi_srs_generate": ([vp, vp, u8p, pp], c_int),
        "mi_srs_export_vk": ([vp, vp, vp], c_int),
        "mi_srs_export_query": ([vp, vp, c_int, vp, u64], c_int),
        "mi_srs_info": ([vp, vp], c_int),
        "mi_srs_free": ([vp], None),
        "mi_srs_msm_info": ([vp, vp], c_int),
        "mi_srs_table_state": ([vp, vp], c_int),
        "mi_srs_readmit": ([vp, vp, vp], c_int),
        "mi_ctx_inject_oom": ([vp, ctypes.c_int64], c_int),
        "mi_tune_set": ([u8p, ctypes.c_int64], c_int),
        "mi_fq_check_read": ([vp, c_int], c_int),
        "mi_tune_clear": ([u8p], c_int),
        "mi_tune_get": ([u8p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(c_int)], c_int),
        "mi_param_cache_id": ([u8p, u8p, vp, ctypes.c_size_t], c_int),
        "mi_param_cache_path": ([u8p, c_int, vp, ctypes.c_size_t], c_int),
        "mi_param_cache_metadata": ([u8p, u64, vp], c_int),
        "mi_get_groth_params": ([vp, vp, u8p, vp, c_int, pp, ctypes.POINTER(c_int)], c_int),
        "mi_groth16_h_coeffs_dev": ([vp, vp, vp, vp], c_int),
        "mi_groth16_prove_share_ranges_h_dev": ([vp, vp, vp, vp, vp, vp, c_int, vp], c_int),
        "mi_stacked_build": ([vp, c_int, pp], c_int),
        "mi_post_build": ([vp, c_int, pp], c_int),
        "mi_stacked_load": ([vp, vp, pp], c_int),
        "mi_stacked_info": ([vp, vp], c_int),
        "mi_stacked_r1cs": ([vp, vp], c_int),
        "mi_stacked_public_inputs": ([vp, vp, vp], c_int),
        "mi_stacked_witness_dev": ([vp, vp, vp, vp], c_int),
        "mi_stacked_witness": ([vp, vp, vp, vp], c_int),
        "mi_stacked_free": ([vp], None),
        "mi_circuit_check_dev": ([vp, vp, vp, vp], c_int),
        "mi_srs_stream_begin": ([vp, vp, u8p, u8p, u64, vp, c_int, pp], c_int),
        "mi_srs_stream_part": ([vp, c_int, u64, vp, u64, c_int], c_int),
        "mi_srs_stream_end": ([vp, pp], c_int),
        "mi_srs_stream_abort": ([vp], None),
        "mi_srs_export_query_dev": ([vp, vp, c_int, u64, u64, vp], c_int),
        "mi_groth16_prove_random": ([vp, vp, vp, u8p, c_int, vp], c_int),
        "mi_groth16_prove_dev_random": ([vp, vp, vp, vp, c_int, vp], c_int),
        "mi_groth16_prove_batch_random": ([vp, vp, vp, u64, vp, c_int, vp], c_int),
        "mi_points_check_subgroup": ([vp, vp], c_int),
        "mi_points_info": ([vp, vp], c_int),
        "mi_points_precompute": ([vp, vp, ctypes.c_uint, ctypes.c_uint64], c_int),
        "mi_points_table_info": ([vp, vp], c_int),
        "mi_ctx_get_table_msms": ([vp, vp], c_int),
        "mi_srs_window_tables": ([vp, vp], c_int),
        "mi_srs_shared_la": ([vp, ctypes.POINTER(c_int)], c_int),
        "mi_ctx_get_shared_plans": ([vp, ctypes.POINTER(ctypes.c_uint64)], c_int),
        "mi_ctx_get_derived_plans": ([vp, ctypes.POINTER(ctypes.c_uint64)], c_int),
        "mi_groth16_prove": ([vp, vp, vp, u8p, u8p, u8p, c_int, vp, vp], c_int),
        "mi_groth16_prove_dev": ([vp, vp, vp, vp, u8p, u8p, c_int, vp, vp], c_int),
        "mi_groth16_prove_batch": ([vp, vp, vp, u64, vp, u8p, c_int, vp], c_int),
        "mi_groth16_prove_share": ([vp, vp, vp, u8p, ctypes.c_uint32, ctypes.c_uint32, c_int, vp], c_int),
        "mi_groth16_prove_share_dev": ([vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, c_int, vp], c_int),
        "mi_groth16_prove_share_ranges": ([vp, vp, vp, vp, vp, c_int, vp], c_int),
        "mi_groth16_prove_share_ranges_dev": ([vp, vp, vp, vp, vp, c_int, vp], c_int),
        "mi_groth16_assemble": ([u8p, u8p, u64, u8p, u8p, vp, vp], c_int),
        "mi_groth16_trapdoor_dlogs": ([vp, vp, vp, vp, u8p, u8p, vp], c_int),
        "mi_msm_g1": ([vp, u8p, u8p, u64, vp], c_int),
        "mi_msm_g2": ([vp, u8p, u8p, u64, vp], c_int),
        "mi_ntt_fr": ([vp, vp, ctypes.c_uint, c_int, c_int], c_int),
        "mi_points_upload_g1": ([vp, u8p, u64, pp], c_int),
        "mi_points_upload_g2": ([vp, u8p, u64, pp], c_int),
        "mi_points_from_srs": ([vp, vp, c_int, pp], c_int),
        "mi_points_free": ([vp], None),
        "mi_points_count": ([vp], u64),
        "mi_msm_g1_dev": ([vp, vp, vp, u64, vp], c_int),
        "mi_msm_g2_dev": ([vp, vp, vp, u64, vp], c_int),
        "mi_ntt_fr_dev": ([vp, vp, ctypes.c_uint, c_int, c_int], c_int),
        "mi_ctx_get_stats": ([vp, vp], c_int),
        "mi_ctx_reset_stats": ([vp], c_int),
        "mi_ctx_get_work": ([vp, vp], c_int),
        "mi_ctx_get_fallbacks": ([vp, vp], c_int),
        "mi_msm_window_bits": ([u64], ctypes.c_uint),
        "mi_synth_generate": ([ctypes.c_uint, u64, u64, pp], c_int),
        "mi_synth_generate_ex": ([ctypes.c_uint, u64, u64, ctypes.c_uint, pp], c_int),
        "mi_synth_r1cs": ([vp, vp], c_int),
        "mi_synth_witness": ([vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u64)], c_int),
        "mi_synth_free": ([vp], None),
        "mi_params_inspect": ([u8p, vp], c_int),
        "mi_params_load": ([vp, vp, u8p, c_int, pp], c_int),
        "mi_params_write": ([vp, vp, u8p], c_int),
        "mi_vk_write": ([vp, u8p], c_int),
        "mi_groth16_verify": ([u8p, u8p, u64, u8p, u8p, ctypes.POINTER(c_int)], c_int),
        "mi_groth16_verify_batch": ([u8p, u8p, u64, u64, u8p, u8p, ctypes.POINTER(c_int)], c_int),
        "mi_groth16_verify_batch_seeded": ([u8p, u8p, u64, u64, u8p, u8p, u8p, ctypes.POINTER(c_int)], c_int),
        "mi_host_alloc": ([u64, pp], c_int),
        "mi_host_free": ([vp], None),
        "mi_pairing": ([u8p, u8p, vp], c_int),
        "mi_poseidon_constants": ([ctypes.c_uint, vp, vp, vp], c_int),
        "mi_poseidon_hash": ([vp, ctypes.c_uint, vp, u64, vp], c_int),
        "mi_poseidon_hash_dev": ([vp, ctypes.c_uint, vp, u64, vp], c_int),
        "mi_tree_cache_size": ([u64, ctypes.c_uint, ctypes.c_uint, vp], c_int),
        "mi_tree_build": ([vp, ctypes.c_uint, vp, u64, ctypes.c_uint, vp], c_int),
        "mi_tree_build_dev": ([vp, ctypes.c_uint, vp, u64, ctypes.c_uint, vp], c_int),
        "mi_tree_c_build": ([vp, ctypes.c_uint, u64, vp, ctypes.c_uint, vp, vp], c_int),
        "mi_tree_c_build_dev": ([vp, ctypes.c_uint, u64, vp, ctypes.c_uint, vp, vp], c_int),
        "mi_tree_r_last_build": ([vp, u64, vp, vp, ctypes.c_uint, ctypes.c_uint, vp], c_int),
        "mi_tree_r_last_build_dev": ([vp, u64, vp, vp, ctypes.c_uint, ctypes.c_uint, vp], c_int),
        "mi_tree_inclusion_paths_dev": ([vp, ctypes.c_uint, vp, u64, ctypes.c_uint, vp, u64, vp, vp, vp], c_int),
        "mi_tree_d_inclusion_paths_dev": ([vp, vp, u64, vp, u64, vp, vp, vp], c_int),
        "mi_tree_d_build_dev": ([vp, vp, u64, vp], c_int),
        "mi_sdr_labels": ([vp, vp, u64, vp, vp, vp, ctypes.c_uint, vp], c_int),
        "mi_sdr_labels_dev": ([vp, vp, u64, vp, vp, vp, ctypes.c_uint, vp], c_int),
        "mi_sdr_labeling_proofs_dev": ([vp, vp, ctypes.c_uint, u64, vp, u64, vp, vp, vp, ctypes.c_uint,
                                        ctypes.c_uint, vp, vp], c_int),
    }
    missing = []
    for name, (args, res) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:  # an older build (same-box A/B of library variants): fails when called
            missing.append(name)
            continue
        f.argtypes = args
        f.restype = res
    L.missing_symbols = missing
    _lib = L
    return L


def check(rc):
    if rc != 0:
        msg = lib().mi_last_error()
        raise FilGpuError(rc, msg.decode() if msg else "")
    return rc
