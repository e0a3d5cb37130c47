"""ctypes binding of the engine's C ABI (include/mimic_amd.h) -> mimic_amd/libmimic_amd.so.

The shared library is built in-tree by ``__graft_entry__.build()``.  There is no fallback:
if the library is missing the import fails loudly (the product path never runs on CPU).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MIMIC_LIB=<file name>: another in-tree build of the same sources (measurement builds, A/B runs)
LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ.get("MIMIC_LIB", "libmimic_amd.so")))

ABI_VERSION = 4

# status codes (enum mimic_status)
STATUS_NAMES = [
    "OK", "ERR_PC_OOB", "ERR_UNSUPPORTED_OP", "ERR_MEM_UNRESOLVED", "ERR_MEM_NOT_VMMEM",
    "ERR_MEM_BOUNDS", "ERR_MEM_NOT_DATASEC", "ERR_R10_WRITE", "ERR_HELPER_MAP_PTR",
    "ERR_HELPER_KEY", "ERR_HELPER_VALUE", "ERR_HELPER_MAP_OP", "ERR_HELPER_TAILCALL",
    "ERR_HELPER_UNIMPLEMENTED", "ERR_HELPER_CANT_EMULATE", "ERR_LDABS", "PANIC_DIV0",
    "PANIC_SHIFT", "PANIC_BADREG", "PANIC_CALLX", "PANIC_PC", "PANIC_HELPER_NEG",
    "ERR_STEP_LIMIT", "ERR_CALL_DEPTH", "ERR_ENGINE_HELPER", "ERR_NO_CPU", "ERR_CTX_ACCESS", "PANIC_SLICE",
    "ERR_CTX_LOAD", "ERR_CANCELED", "ERR_DEADLINE", "ERR_ENGINE_STATE",
]
STATUS = {n: i for i, n in enumerate(STATUS_NAMES)}
ECANCELED, EDEADLINE = -7, -8   # mimic_process_run_ctx: ctx.Err() (include/mimic_amd.h)

SCHED_CHUNKED, SCHED_INTERLEAVED, SCHED_EXPLICIT = 0, 1, 2
MAP_F_DATASEC = 1


class VMSettings(C.Structure):
    _fields_ = [("vcpus", C.c_int32), ("stack_frame_size", C.c_int32), ("stack_frame_count", C.c_int32),
                ("max_tail_calls", C.c_int32), ("device", C.c_int32), ("vcpu_begin", C.c_int32),
                ("vcpu_count", C.c_int32), ("exec_mode", C.c_int32)]


class MapSpecC(C.Structure):
    _fields_ = [("name", C.c_char_p), ("type", C.c_uint32), ("key_size", C.c_uint32),
                ("value_size", C.c_uint32), ("max_entries", C.c_uint32), ("flags", C.c_uint32)]


class ProcessRegs(C.Structure):
    _fields_ = [("r", C.c_uint64 * 11), ("pc", C.c_int32), ("prog_id", C.c_uint32), ("steps", C.c_uint64),
                ("status", C.c_int32), ("exited", C.c_uint32)]


class Reloc(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("map_id", C.c_uint32)]


class XDPBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("schedule", C.c_uint32), ("pkt_data", C.c_void_p),
                ("pkt_off", C.c_void_p), ("pkt_len", C.c_void_p),
                ("headroom", C.c_void_p), ("headroom_all", C.c_uint32),
                ("tailroom", C.c_void_p), ("tailroom_all", C.c_uint32),
                ("ingress_ifindex", C.c_void_p), ("ingress_all", C.c_int32),
                ("rx_queue_index", C.c_void_p), ("rxq_all", C.c_int32),
                ("egress_ifindex", C.c_void_p), ("egress_all", C.c_int32),
                ("cpu", C.c_void_p), ("step_budget", C.c_uint64)]


class SKBBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("schedule", C.c_uint32), ("pkt_data", C.c_void_p),
                ("pkt_off", C.c_void_p), ("pkt_len", C.c_void_p), ("ifindex", C.c_uint32), ("pad", C.c_int32),
                ("cpu", C.c_void_p), ("step_budget", C.c_uint64), ("custom", C.c_void_p), ("rooms_state", C.c_void_p)]


# mimic_skb_custom (include/mimic_amd.h): a user-given sock / flow keys of one sk_buff context
SKB_CUSTOM_SK, SKB_CUSTOM_FLOWKEYS = 1, 2
try:
    import numpy as _np

    SKB_CUSTOM_DTYPE = _np.dtype([
        ("flags", "<u4"), ("sk_bound_dev_if", "<u4"), ("sk_family", "<u4"), ("sk_type", "<u4"), ("sk_protocol", "<u4"),
        ("sk_mark", "<u4"), ("sk_priority", "<u4"), ("sk_src_port", "<u4"), ("sk_dst_port", "<u4"), ("sk_state", "<u4"),
        ("sk_rx_queue_mapping", "<i4"), ("sk_ip_len", "u1", (4,)), ("sk_ip", "u1", (4, 16)),
        ("fk_nhoff", "<u2"), ("fk_thoff", "<u2"), ("fk_addr_proto", "<u2"), ("fk_is_frag", "u1"),
        ("fk_is_first_frag", "u1"), ("fk_is_encap", "u1"), ("fk_ip_proto", "u1"), ("fk_n_proto", "<u2"),
        ("fk_sport", "<u2"), ("fk_dport", "<u2"), ("fk_flags", "<u4"), ("fk_flow_label", "<u4")])
    assert SKB_CUSTOM_DTYPE.itemsize == 136
except ImportError:   # numpy is a dependency of every batch path; the ABI loads without it
    SKB_CUSTOM_DTYPE = None


CTX_XDP, CTX_SKB = 0, 1


class XDPResults(C.Structure):
    _fields_ = [("r0", C.c_void_p), ("status", C.c_void_p), ("steps", C.c_void_p), ("err_pc", C.c_void_p)]


class XDPHostBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("schedule", C.c_uint32), ("pkt_data", C.c_void_p),
                ("pkt_off", C.c_void_p), ("pkt_len", C.c_void_p),
                ("headroom_all", C.c_uint32), ("tailroom_all", C.c_uint32),
                ("ingress_all", C.c_int32), ("rxq_all", C.c_int32), ("egress_all", C.c_int32), ("pad", C.c_int32),
                ("cpu", C.c_void_p), ("step_budget", C.c_uint64), ("pkt_out", C.c_void_p),
                ("r0", C.c_void_p), ("status", C.c_void_p)]


EXPORTS = {
    "mimic_abi_version": (C.c_int, []),
    "mimic_last_error": (C.c_char_p, [C.c_void_p]),
    "mimic_vm_create": (C.c_int, [C.POINTER(VMSettings), C.POINTER(C.c_void_p)]),
    "mimic_vm_destroy": (None, [C.c_void_p]),
    "mimic_map_create": (C.c_int, [C.c_void_p, C.POINTER(MapSpecC), C.POINTER(C.c_uint32)]),
    "mimic_map_update": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int32]),
    "mimic_map_lookup": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int32, C.POINTER(C.c_uint32)]),
    "mimic_map_update_batch": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                         C.c_int32, C.c_void_p]),
    "mimic_map_delete": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "mimic_exec_mode": (C.c_int, [C.c_void_p]),
    "mimic_set_spread": (C.c_int, [C.c_void_p, C.c_int32]),
    "mimic_process_new_skb_ctx": (C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                            C.POINTER(C.c_void_p)]),
    "mimic_run_xdp_host": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(XDPHostBatch), C.c_uint32]),
    "mimic_host_register": (C.c_int, [C.c_void_p, C.c_size_t]),
    "mimic_host_unregister": (C.c_int, [C.c_void_p]),
    "mimic_last_exec": (C.c_int, [C.c_void_p]),
    "mimic_jit_source_for": (C.c_long, [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_char_p,
                                         C.c_size_t]),
    "mimic_jit_check": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "mimic_jit_prebuild": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32]),
    "mimic_map_keys": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint32)]),
    "mimic_map_entries": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_size_t,
                                    C.POINTER(C.c_uint32)]),
    "mimic_map_read_values": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.c_void_p, C.c_size_t]),
    "mimic_map_reset": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "mimic_map_read_values_range": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_void_p, C.c_size_t]),
    "mimic_map_sum_u64": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_void_p, C.c_size_t]),
    "mimic_map_addr": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "mimic_program_load": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.POINTER(Reloc),
                                     C.c_uint32, C.POINTER(C.c_uint32)]),
    "mimic_program_addr": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "mimic_mem_read": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    "mimic_mem_load": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int32, C.POINTER(C.c_uint64)]),
    "mimic_stack_addr": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "mimic_run_xdp": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(XDPBatch), C.POINTER(XDPResults), C.c_void_p]),
    "mimic_run_xdp_many": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(XDPBatch), C.POINTER(XDPResults), C.c_uint32,
                                     C.c_void_p]),
    "mimic_map_share": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    "mimic_run_skb": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(SKBBatch), C.POINTER(XDPResults), C.c_void_p]),
    "mimic_skb_release": (C.c_int, [C.c_void_p]),
    "mimic_jit_source_for_ctx": (C.c_long, [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_int32,
                                             C.c_char_p, C.c_size_t]),
    "mimic_jit_source_vc": (C.c_long, [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_int32,
                                       C.POINTER(C.c_uint32), C.c_uint32, C.c_char_p, C.c_size_t]),
    "mimic_jit_source_spread": (C.c_long, [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32,
                                           C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32,
                                           C.c_uint32, C.POINTER(C.c_int32), C.c_char_p, C.c_size_t]),
    "mimic_jit_prebuild_ctx": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_int32]),
    "mimic_jit_cache_source": (C.c_int, [C.c_char_p]),
    "mimic_process_new": (C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "mimic_process_new_skb": (C.c_int, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_uint32, C.c_uint32, C.c_void_p]),
    "mimic_process_set_cpu": (C.c_int, [C.c_void_p, C.c_int32]),
    "mimic_process_step": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "mimic_process_run": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p]),
    "mimic_process_packet": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "mimic_process_free": (None, [C.c_void_p]),
    "mimic_jit_code": (C.c_int, [C.c_char_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "mimic_sync": (C.c_int, [C.c_void_p, C.c_void_p]),
    "mimic_ctx_new": (C.c_int, [C.c_uint64, C.POINTER(C.c_void_p)]),
    "mimic_ctx_cancel": (None, [C.c_void_p]),
    "mimic_ctx_err": (C.c_int, [C.c_void_p]),
    "mimic_ctx_pinned": (C.c_int, [C.c_void_p]),
    "mimic_ctx_free": (None, [C.c_void_p]),
    "mimic_run_xdp_ctx": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(XDPBatch), C.POINTER(XDPResults), C.c_void_p,
                                    C.c_void_p, C.c_void_p]),
    "mimic_run_skb_ctx": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(SKBBatch), C.POINTER(XDPResults), C.c_void_p,
                                    C.c_void_p, C.c_void_p]),
    "mimic_process_run_ctx": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.POINTER(ProcessRegs)]),
    "mimic_process_run_many": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(ProcessRegs)]),
    "mimic_process_free_many": (None, [C.c_void_p, C.c_uint32]),
    "mimic_run_xdp_host_ctx": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(XDPHostBatch), C.c_uint32, C.c_void_p]),
    "mimic_run_xdp_host_ctx_pp": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(XDPHostBatch), C.c_uint32, C.c_void_p]),
    "mimic_last_steps": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
}

_lib = None


def load() -> C.CDLL:
    """Load libmimic_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    # torch's wheel bundles its own ROCm runtime (libamdhip64 / libhiprtc / comgr).  torch links it
    # by a name the engine's NEEDED entry does not match, so loading the engine first would put two
    # HIP runtimes in the process; loading torch first lets the engine bind to torch's copy by
    # soname: one runtime, one device context, shared by the engine's kernels and torch's tensors.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mimic_abi_version() != ABI_VERSION:
        raise ImportError("libmimic_amd.so ABI version mismatch")
    _lib = lib
    return lib
