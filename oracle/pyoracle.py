"""ctypes wrapper of the C oracle (test infrastructure only)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MIMIC_ORACLE_LIB: another build of the same source (tools/run_asan.sh: the sanitizer build)
LIB_PATH = os.environ.get("MIMIC_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")


class OracleError(RuntimeError):
    pass


class _Reloc(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("map_id", C.c_uint32)]


class _Batch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("pkt_data", C.c_void_p), ("pkt_off", C.c_void_p), ("pkt_len", C.c_void_p),
                ("headroom_arr", C.c_void_p), ("headroom", C.c_uint32), ("tailroom_arr", C.c_void_p),
                ("tailroom", C.c_uint32), ("ingress_ifindex", C.c_void_p), ("rx_queue_index", C.c_void_p),
                ("egress_ifindex", C.c_void_p), ("cpu", C.c_void_p), ("step_budget", C.c_uint64),
                ("write_back", C.c_int), ("ctx_done", C.c_void_p), ("ctx_done_step", C.c_void_p)]


class _SkbBatch(C.Structure):
    _fields_ = [("n", C.c_uint32), ("pkt_data", C.c_void_p), ("pkt_off", C.c_void_p), ("pkt_len", C.c_void_p),
                ("ifindex", C.c_uint32), ("cpu", C.c_void_p), ("step_budget", C.c_uint64), ("write_back", C.c_int),
                ("custom", C.c_void_p), ("ctx_done", C.c_void_p), ("ctx_done_step", C.c_void_p)]


class _Results(C.Structure):
    _fields_ = [("r0", C.c_void_p), ("status", C.c_void_p), ("steps", C.c_void_p), ("err_pc", C.c_void_p)]


_lib = None


def load(build: bool = True) -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build:
            raise OracleError(f"{LIB_PATH} missing")
        subprocess.check_call(["make", "-C", _HERE, "-s"])
    lib = C.CDLL(LIB_PATH)
    sig = {
        "orc_vm_new": (C.c_void_p, [C.c_int, C.c_int, C.c_int, C.c_int]),
        "orc_vm_free": (None, [C.c_void_p]),
        "orc_last_error": (C.c_char_p, [C.c_void_p]),
        "orc_map_create": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int]),
        "orc_map_update": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int]),
        "orc_map_lookup": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_uint32)]),
        "orc_map_delete": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
        "orc_map_values": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_size_t]),
        "orc_map_slots": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]),
        "orc_map_addr": (C.c_uint32, [C.c_void_p, C.c_int]),
        "orc_prog_load": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
        "orc_prog_addr": (C.c_uint32, [C.c_void_p, C.c_int]),
        "orc_mem_add_scratch": (C.c_uint32, [C.c_void_p, C.c_uint32]),
        "orc_mem_read": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
        "orc_mem_write": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
        "orc_mem_load": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int, C.POINTER(C.c_uint64)]),
        "orc_mem_next_free": (C.c_uint32, [C.c_void_p]),
        "orc_proc_new": (C.c_void_p, [C.c_void_p, C.c_int]),
        "orc_proc_free": (None, [C.c_void_p]),
        "orc_proc_set_cpu": (C.c_int, [C.c_void_p, C.c_int]),
        "orc_proc_get_reg": (C.c_uint64, [C.c_void_p, C.c_int]),
        "orc_proc_set_reg": (None, [C.c_void_p, C.c_int, C.c_uint64]),
        "orc_proc_call_helper": (C.c_int, [C.c_void_p, C.c_int32]),
        "orc_proc_new_xdp": (C.c_void_p, [C.c_void_p, C.c_int, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_int32, C.c_int32, C.c_int32]),
        "orc_proc_new_skb_ctx": (C.c_void_p, [C.c_void_p, C.c_int, C.c_char_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                              C.POINTER(C.c_int)]),
        "orc_proc_new_skb": (C.c_void_p, [C.c_void_p, C.c_int, C.c_char_p, C.c_uint32, C.c_uint32,
                                          C.POINTER(C.c_int)]),
        "orc_proc_step": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
        "orc_proc_get_pc": (C.c_int64, [C.c_void_p]),
        "orc_proc_get_prog": (C.c_int, [C.c_void_p]),
        "orc_run_xdp_batch": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(_Batch), C.POINTER(_Results)]),
        "orc_run_skb_batch": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(_SkbBatch), C.POINTER(_Results)]),
    }
    for n, (r, a) in sig.items():
        f = getattr(lib, n)
        f.restype = r
        f.argtypes = a
    _lib = lib
    return lib


class OracleProcess:
    def __init__(self, vm: "OracleVM", prog_id: int, xdp=None, skb=None):
        """xdp = (packet bytes, headroom, tailroom, ingress, rxq, egress): an xdp_md context;
        skb = (packet bytes, ifindex[, custom]): an sk_buff context (Load at construction); custom =
        a numpy orc_skb_custom record (the engine's mimic_skb_custom layout) or None."""
        self.vm = vm
        if skb is not None:
            pkt, ifindex = skb[0], skb[1]
            custom = skb[2] if len(skb) > 2 else None
            st = C.c_int(0)
            self._custom = None if custom is None else np.ascontiguousarray(custom)
            cp = None if self._custom is None else self._custom.ctypes.data
            self.p = vm.lib.orc_proc_new_skb_ctx(vm.h, prog_id, bytes(pkt), len(pkt), ifindex, cp, C.byref(st))
            if not self.p:
                raise OracleError(f"sk_buff context load failed (status {st.value})")
            return
        if xdp is None:
            self.p = vm.lib.orc_proc_new(vm.h, prog_id)
        else:
            pkt, H, T, ing, rxq, eg = xdp
            self.p = vm.lib.orc_proc_new_xdp(vm.h, prog_id, bytes(pkt), len(pkt), H, T, ing, rxq, eg)
        if not self.p:
            raise OracleError("no such program")

    def step(self):
        """Process.Step: (0 continue | -1 exited | status, err_pc)."""
        e = C.c_int32(-1)
        rc = self.vm.lib.orc_proc_step(self.p, C.byref(e))
        return rc, e.value

    def pc(self) -> int:
        return self.vm.lib.orc_proc_get_pc(self.p)

    def prog(self) -> int:
        return self.vm.lib.orc_proc_get_prog(self.p)

    def set_cpu(self, c: int) -> int:
        return self.vm.lib.orc_proc_set_cpu(self.p, c)

    def reg(self, r: int) -> int:
        return self.vm.lib.orc_proc_get_reg(self.p, r)

    def set_reg(self, r: int, v: int) -> None:
        self.vm.lib.orc_proc_set_reg(self.p, r, v & 0xFFFFFFFFFFFFFFFF)

    def call_helper(self, n: int) -> int:
        return self.vm.lib.orc_proc_call_helper(self.p, n)

    def cleanup(self) -> None:
        if self.p:
            self.vm.lib.orc_proc_free(self.p)
            self.p = None


class OracleVM:
    def __init__(self, vcpus: int, stack_frame_size: int = 256, stack_frame_count: int = 8, max_tail_calls: int = 33):
        self.lib = load()
        self.h = self.lib.orc_vm_new(vcpus, stack_frame_size, stack_frame_count, max_tail_calls)
        self.vcpus = vcpus
        self.map_ids = {}
        self.specs = {}

    def close(self):
        if self.h:
            self.lib.orc_vm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def err(self) -> str:
        return (self.lib.orc_last_error(self.h) or b"").decode()

    def map_create(self, name: str, type_: int, key_size: int, value_size: int, max_entries: int,
                   datasec: bool = False) -> int:
        mid = self.lib.orc_map_create(self.h, name.encode(), type_, key_size, value_size, max_entries, int(datasec))
        if mid < 0:
            raise OracleError(self.err())
        self.map_ids[name] = mid
        self.specs[mid] = (type_, key_size, value_size, max_entries)
        return mid

    def map_update(self, mid: int, key: bytes, value: bytes, flags: int = 0, cpu: int = 0) -> int:
        return self.lib.orc_map_update(self.h, mid, bytes(key), bytes(value), flags, cpu)

    def map_lookup(self, mid: int, key: bytes, cpu: int = 0) -> Tuple[int, int]:
        a = C.c_uint32()
        rc = self.lib.orc_map_lookup(self.h, mid, bytes(key), cpu, C.byref(a))
        return rc, a.value

    def map_values(self, mid: int, cpu: int = 0) -> bytes:
        _, _, S, E = self.specs[mid]
        buf = C.create_string_buffer(max(S * E, 1))
        n = self.lib.orc_map_values(self.h, mid, cpu, buf, max(S * E, 1))
        if n < 0:
            raise OracleError("map_values")
        return buf.raw[:n]

    def map_entries(self, mid: int) -> List[Tuple[bytes, int]]:
        """Live (key, slot) pairs of a hash map (KeyToIndex)."""
        _, K, _, E = self.specs[mid]
        sl = (C.c_int32 * max(E, 1))()
        kb = C.create_string_buffer(max(K * E, 1))
        n = self.lib.orc_map_slots(self.h, mid, sl, kb, max(E, 1))
        if n < 0:
            raise OracleError("map_entries")
        raw = kb.raw
        slots = np.frombuffer(sl, np.int32)
        return [(raw[i * K:(i + 1) * K], int(slots[i])) for i in range(n)]

    def map_addr(self, mid: int) -> int:
        return self.lib.orc_map_addr(self.h, mid)

    def prog_load(self, name: str, raw: bytes, relocs: Sequence[Tuple[int, int]] = ()) -> int:
        arr = (_Reloc * max(len(relocs), 1))(*[_Reloc(s, m) for s, m in relocs])
        pid = self.lib.orc_prog_load(self.h, name.encode(), bytes(raw), len(raw) // 8, arr, len(relocs))
        if pid < 0:
            raise OracleError(self.err())
        return pid

    def prog_addr(self, pid: int) -> int:
        return self.lib.orc_prog_addr(self.h, pid)

    def mem_add_scratch(self, size: int) -> int:
        return self.lib.orc_mem_add_scratch(self.h, size)

    def mem_write(self, addr: int, data: bytes) -> int:
        return self.lib.orc_mem_write(self.h, addr, bytes(data), len(data))

    def mem_read(self, addr: int, n: int) -> Optional[bytes]:
        buf = C.create_string_buffer(max(n, 1))
        rc = self.lib.orc_mem_read(self.h, addr, buf, n)
        return None if rc else buf.raw[:n]

    def mem_load(self, addr: int, size: int) -> Tuple[int, int]:
        v = C.c_uint64()
        rc = self.lib.orc_mem_load(self.h, addr, size, C.byref(v))
        return rc, v.value

    def next_free(self) -> int:
        return self.lib.orc_mem_next_free(self.h)

    def new_process(self, prog_id: int) -> OracleProcess:
        return OracleProcess(self, prog_id)

    def run_xdp_batch(self, prog_id: int, buf: np.ndarray, off: np.ndarray, lens: np.ndarray, cpu: np.ndarray,
                      headroom=0, tailroom=0, ingress=None, rxq=None, egress=None, step_budget: int = 0,
                      write_back: bool = True, ctx_done=None, ctx_done_step=None):
        """Sequential reference run over a numpy packet buffer (modified in place if write_back).
        ctx_done: None, or per packet the state of its Run's ctx (0 not done, 1 canceled, 2
        deadline exceeded; orc_xdp_batch.ctx_done); ctx_done_step: per packet, the step before
        which its ctx is seen done (None: before the first)."""
        n = len(lens)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        cpu = np.ascontiguousarray(cpu, dtype=np.int32)
        keep = []

        def arr(v, dt):
            if v is None or np.isscalar(v):
                return None
            a = np.ascontiguousarray(v, dtype=dt)
            keep.append(a)
            return a.ctypes.data

        b = _Batch()
        b.n = n
        b.pkt_data = buf.ctypes.data
        b.pkt_off = off.ctypes.data
        b.pkt_len = lens.ctypes.data
        b.headroom_arr = arr(headroom, np.uint32)
        b.headroom = int(headroom) if np.isscalar(headroom) else 0
        b.tailroom_arr = arr(tailroom, np.uint32)
        b.tailroom = int(tailroom) if np.isscalar(tailroom) else 0
        b.ingress_ifindex = arr(ingress, np.int32)
        b.rx_queue_index = arr(rxq, np.int32)
        b.egress_ifindex = arr(egress, np.int32)
        b.cpu = cpu.ctypes.data
        b.step_budget = step_budget
        b.write_back = int(write_back)
        b.ctx_done = arr(ctx_done, np.uint8)
        b.ctx_done_step = arr(ctx_done_step, np.uint32)
        out = {"r0": np.zeros(n, np.uint64), "status": np.zeros(n, np.uint8), "steps": np.zeros(n, np.uint32),
               "err_pc": np.zeros(n, np.int32)}
        r = _Results(out["r0"].ctypes.data, out["status"].ctypes.data, out["steps"].ctypes.data,
                     out["err_pc"].ctypes.data)
        rc = self.lib.orc_run_xdp_batch(self.h, prog_id, C.byref(b), C.byref(r))
        if rc:
            raise OracleError(self.err())
        out["pkt"] = buf
        return out

    def run_skb_batch(self, prog_id: int, buf: np.ndarray, off: np.ndarray, lens: np.ndarray, cpu: np.ndarray,
                      ifindex: int = 0, step_budget: int = 0, write_back: bool = True, custom=None, ctx_done=None,
                      ctx_done_step=None):
        """Sequential sk_buff-context run: packet i is lens[i] bytes at buf[off[i] + 32:]; the
        process's packet memory [off[i], off[i] + 96 + L) is written back if write_back.  custom:
        a numpy table of orc_skb_custom records (one per packet) or None."""
        n = len(lens)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        cpu = np.ascontiguousarray(cpu, dtype=np.int32)
        cu = None if custom is None else np.ascontiguousarray(custom)
        if cu is not None:
            assert cu.dtype.itemsize == 136 and len(cu) == n
        cd = None if ctx_done is None else np.ascontiguousarray(ctx_done, dtype=np.uint8)
        cs = None if ctx_done_step is None else np.ascontiguousarray(ctx_done_step, dtype=np.uint32)
        b = _SkbBatch(n, buf.ctypes.data, off.ctypes.data, lens.ctypes.data, ifindex, cpu.ctypes.data, step_budget,
                      int(write_back), None if cu is None else cu.ctypes.data, None if cd is None else cd.ctypes.data,
                      None if cs is None else cs.ctypes.data)
        out = {"r0": np.zeros(n, np.uint64), "status": np.zeros(n, np.uint8), "steps": np.zeros(n, np.uint32),
               "err_pc": np.zeros(n, np.int32)}
        r = _Results(out["r0"].ctypes.data, out["status"].ctypes.data, out["steps"].ctypes.data,
                     out["err_pc"].ctypes.data)
        if self.lib.orc_run_skb_batch(self.h, prog_id, C.byref(b), C.byref(r)):
            raise OracleError(self.err())
        out["pkt"] = buf
        return out
