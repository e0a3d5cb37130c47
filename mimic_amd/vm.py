"""Python mirror of mimic's Go surface for the Process.Run hot path, backed by the C ABI.

Reference names are kept so parity tests read like the reference's own tests
(emulator_linux_helpers_test.go, emulator_linux_map_array_test.go):

    emu = NewLinuxEmulator()                                 # emulator_linux_.go:67
    vm = NewVM(VMOptEmulator(emu), VMOptSetvCPUs(2))         # vm.go:54
    m = LinuxPerCPUArrayMap(Spec=MapSpec(...))               # emulator_linux_map_array.go:177
    emu.AddMap("per-cpu-array", m)                           # emulator_linux_.go:97
    m.Update(key, value, 0, CPU0); addr = m.Lookup(key, CPU0)
    vm.MemoryController.GetEntry(addr) / .Load(addr, 4)     # memory_controller.go:117
    prog_id = vm.AddProgram(ProgramSpec(...))                # vm.go:98
    p = vm.NewProcess(prog_id, LinuxContextXDP(Packet=...)) # vm.go:198 + context_xdp_md.go:47
    p.SetCPUID(0); p.Run(); p.Registers.R0; p.Cleanup()      # vm.go:268,343,363

plus the batch entry point the GPU exists for:

    res = vm.RunXDPBatch(prog_id, XDPBatch.from_packets([...]))   # N processes at once

Errors follow the reference: a graceful map error is a ``syscall.Errno``-like positive int
(E2BIG = 7) returned by Update; fatal errors raise ``MimicError``.
"""
from __future__ import annotations

import base64
import ctypes as C
import json
import os
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from . import _lib as L


class MimicError(RuntimeError):
    pass


class MapType(IntEnum):  # ebpf.MapType (cilium/ebpf v0.9.0; kernel numbering)
    Hash = 1
    Array = 2
    ProgramArray = 3
    PerfEventArray = 4
    PerCPUHash = 5
    PerCPUArray = 6


E2BIG = 7


@dataclass
class MapSpec:  # ebpf.MapSpec (the fields the emulator reads)
    Name: str
    Type: int
    KeySize: int
    ValueSize: int
    MaxEntries: int
    Datasec: bool = False  # Spec.Value is a *btf.Datasec


@dataclass
class ProgramSpec:  # ebpf.ProgramSpec: raw instruction slots + map references
    Name: str
    Instructions: bytes
    References: List[Tuple[int, str]] = field(default_factory=list)  # (slot, map name)


def _check(vm_handle, rc: int, what: str) -> int:
    if rc < 0:
        lib = L.load()
        msg = lib.mimic_last_error(vm_handle) if vm_handle else b""
        raise MimicError(f"{what}: {msg.decode(errors='replace') if msg else rc}")
    return rc


# ---------------------------------------------------------------------------------------------
# emulator + maps
# ---------------------------------------------------------------------------------------------

def OptMaxTailCalls(n: int):
    return ("max_tail_calls", n)


class LinuxEmulator:
    """emulator_linux_.go:55-64.  Maps are created on the device when the emulator is attached
    to a VM (the reference's Init needs the VM's memory controller too, vm.go:73)."""

    def __init__(self, MaxTailCalls: int = 33):
        self.MaxTailCalls = MaxTailCalls
        self.Maps: Dict[str, "LinuxMap"] = {}
        self.vm: Optional["VM"] = None

    def SetVM(self, vm: "VM") -> None:  # emulator_linux_.go:120-122
        self.vm = vm

    def AddMap(self, name: str, m: "LinuxMap") -> None:  # emulator_linux_.go:97-116
        if self.vm is None:
            raise MimicError("emulator is not attached to a VM")
        if name in self.Maps:
            raise MimicError(f"map with name '{name}' already exists in emulator")
        m.Init(self)
        self.Maps[name] = m


def NewLinuxEmulator(*opts) -> LinuxEmulator:
    emu = LinuxEmulator()
    for k, v in opts:
        setattr(emu, {"max_tail_calls": "MaxTailCalls"}[k], v)
    return emu


class LinuxMap:
    """Common LinuxMap surface (emulator_linux_map.go:14-54) over a device-resident map."""

    def __init__(self, Spec: MapSpec):
        self.Spec = Spec
        self.id: Optional[int] = None
        self.emulator: Optional[LinuxEmulator] = None

    # LinuxMap.Init
    def Init(self, emulator: LinuxEmulator) -> None:
        vm = emulator.vm
        spec = L.MapSpecC(self.Spec.Name.encode(), int(self.Spec.Type), self.Spec.KeySize, self.Spec.ValueSize,
                          self.Spec.MaxEntries, L.MAP_F_DATASEC if self.Spec.Datasec else 0)
        mid = C.c_uint32()
        _check(vm.h, vm.lib.mimic_map_create(vm.h, C.byref(spec), C.byref(mid)), "map init")
        self.id = mid.value
        self.emulator = emulator

    @property
    def _vm(self) -> "VM":
        return self.emulator.vm

    def GetSpec(self) -> MapSpec:
        return self.Spec

    def Indices(self) -> int:
        return 1

    def Lookup(self, key: bytes, cpuid: int = 0) -> int:
        """Virtual address of the value, 0 if absent (LinuxMap.Lookup)."""
        vm = self._vm
        if len(key) != self.Spec.KeySize:
            raise MimicError("size of given key doesn't match key size in map spec")
        addr = C.c_uint32()
        _check(vm.h, vm.lib.mimic_map_lookup(vm.h, self.id, bytes(key), cpuid, C.byref(addr)), "lookup")
        return addr.value

    def Update(self, key: bytes, value: bytes, flags: int = 0, cpuid: int = 0) -> int:
        """0 on success or a positive errno (graceful, e.g. E2BIG); raises on fatal errors."""
        vm = self._vm
        if len(value) != self.Spec.ValueSize:
            raise MimicError(f"invalid value length, must be {self.Spec.ValueSize} bytes")
        if len(key) != self.Spec.KeySize:   # emulator_linux_map_hash.go:159-161, _array.go:98-100
            raise MimicError("size of given key doesn't match key size in map spec")
        rc = vm.lib.mimic_map_update(vm.h, self.id, bytes(key), bytes(value), flags, cpuid)
        return rc if rc >= 0 else _check(vm.h, rc, "update")

    def UpdateBatch(self, keys, values, flags: int = 0, cpuid: int = 0):
        """Not in the reference API: Update(keys[i], values[i]) for every i in one call (numpy
        uint8 arrays of shape (n, KeySize) / (n, ValueSize), or concatenated bytes).  Returns the
        per-call results (0 or a positive errno) as a numpy int32 array."""
        import numpy as np

        vm = self._vm
        kb = np.ascontiguousarray(np.frombuffer(keys, np.uint8) if isinstance(keys, (bytes, bytearray)) else keys,
                                  dtype=np.uint8).reshape(-1)
        vb = np.ascontiguousarray(np.frombuffer(values, np.uint8) if isinstance(values, (bytes, bytearray)) else values,
                                  dtype=np.uint8).reshape(-1)
        n = len(kb) // max(self.Spec.KeySize, 1)
        if len(kb) != n * self.Spec.KeySize or len(vb) != n * self.Spec.ValueSize:
            raise MimicError("keys / values do not hold the same number of entries")
        rcs = np.zeros(n, np.int32)
        _check(vm.h, vm.lib.mimic_map_update_batch(vm.h, self.id, kb.ctypes.data, vb.ctypes.data, n, flags, cpuid,
                                                   rcs.ctypes.data), "update batch")
        return rcs

    def Delete(self, key: bytes) -> int:
        vm = self._vm
        if len(key) != self.Spec.KeySize:
            raise MimicError("size of given key doesn't match key size in map spec")
        return _check(vm.h, vm.lib.mimic_map_delete(vm.h, self.id, bytes(key)), "delete")

    def Values(self, cpuid: int = 0) -> bytes:
        """Raw value backing (MaxEntries * ValueSize bytes) of one cpu."""
        vm = self._vm
        n = self.Spec.MaxEntries * self.Spec.ValueSize
        buf = C.create_string_buffer(max(n, 1))
        _check(vm.h, vm.lib.mimic_map_read_values(vm.h, self.id, cpuid, buf, max(n, 1)), "read values")
        return buf.raw[:n]

    def Share(self, owner: "LinuxMap") -> None:
        """This map (of another VM) becomes ONE table with `owner` (mimic_map_share): inserts, E2BIG,
        lookups and host operations of either VM see the other's.  Not in the reference API."""
        vm, ovm = self._vm, owner._vm
        _check(vm.h, vm.lib.mimic_map_share(vm.h, self.id, ovm.h, owner.id), "share")
        self._share_owner = owner   # the owner's VM must outlive this one

    def Reset(self, stream=None) -> None:
        """Not in the reference API: back to a freshly created map at the same addresses (zeroed
        values, hash maps empty with the freelist 0..E-1), queued on `stream` (mimic_map_reset)."""
        vm = self._vm
        st = stream.cuda_stream if stream is not None else None
        _check(vm.h, vm.lib.mimic_map_reset(vm.h, self.id, st), "reset")

    def ValuesRange(self, cpu_begin: int = 0, cpu_end: Optional[int] = None):
        """Values(c) for every cpu c of [cpu_begin, cpu_end) in one device copy: a numpy uint8 array
        of shape (cpu_end - cpu_begin, MaxEntries * ValueSize)."""
        import numpy as np

        vm = self._vm
        if cpu_end is None:
            cpu_end = self.Indices()
        row = self.Spec.MaxEntries * self.Spec.ValueSize
        out = np.zeros((max(cpu_end - cpu_begin, 0), row), np.uint8)
        _check(vm.h, vm.lib.mimic_map_read_values_range(vm.h, self.id, cpu_begin, cpu_end, out.ctypes.data,
                                                        out.nbytes), "read values range")
        return out

    def SumU64(self, cpu_begin: int = 0, cpu_end: Optional[int] = None) -> List[int]:
        """Per-key sum over vCPUs of a u64-valued map (device reduction)."""
        vm = self._vm
        if cpu_end is None:
            cpu_end = self.Indices()
        out = (C.c_uint64 * self.Spec.MaxEntries)()
        _check(vm.h, vm.lib.mimic_map_sum_u64(vm.h, self.id, cpu_begin, cpu_end, out, self.Spec.MaxEntries),
               "sum")
        return list(out)

    def Address(self) -> int:
        vm = self._vm
        a = C.c_uint32()
        _check(vm.h, vm.lib.mimic_map_addr(vm.h, self.id, C.byref(a)), "map addr")
        return a.value


class LinuxArrayMap(LinuxMap):  # emulator_linux_map_array.go:21-168
    def Keys(self, cpuid: int = 0) -> bytes:
        return b"".join(i.to_bytes(4, "little") for i in range(self.Spec.MaxEntries))

    def UpdateProgram(self, key: bytes, prog_id: int, flags: int = 0) -> int:
        """Store a program's address (what a ProgramArray value holds, read at
        emulator_linux_helpers.go:707)."""
        vm = self._vm
        return self.Update(key, vm.ProgramAddress(prog_id).to_bytes(4, "little"), flags, 0)


class LinuxPerCPUArrayMap(LinuxMap):  # emulator_linux_map_array.go:177-250
    def Indices(self) -> int:
        return self._vm.settings.vcpus

    def Keys(self, cpuid: int = 0) -> bytes:
        return b"".join(i.to_bytes(4, "little") for i in range(self.Spec.MaxEntries))


class LinuxHashMap(LinuxMap):  # emulator_linux_map_hash.go:21-255
    """Exact-key map: a new key takes the head of a FIFO freelist of slots (0..E-1 initially);
    a full freelist is E2BIG; Delete returns the slot to the tail."""

    def _keys(self):
        vm = self._vm
        K, E = self.Spec.KeySize, self.Spec.MaxEntries
        buf = C.create_string_buffer(max(K * E, 1))
        n = C.c_uint32()
        _check(vm.h, vm.lib.mimic_map_keys(vm.h, self.id, buf, max(K * E, 1), C.byref(n)), "keys")
        return buf.raw[:K * n.value], n.value

    def Keys(self, cpuid: int = 0) -> bytes:
        return self._keys()[0]

    def KeyList(self) -> List[bytes]:
        raw, n = self._keys()
        K = self.Spec.KeySize
        return [raw[i * K:(i + 1) * K] for i in range(n)]

    def Entries(self) -> List[Tuple[bytes, int]]:
        """Live (key, slot) pairs (KeyToIndex), table order."""
        vm = self._vm
        K, E = self.Spec.KeySize, self.Spec.MaxEntries
        kb = C.create_string_buffer(max(K * E, 1))
        sl = (C.c_int32 * max(E, 1))()
        n = C.c_uint32()
        _check(vm.h, vm.lib.mimic_map_entries(vm.h, self.id, kb, sl, max(E, 1), C.byref(n)), "entries")
        raw = kb.raw          # one copy of the key buffer (.raw copies on every access)
        return [(raw[i * K:(i + 1) * K], int(s)) for i, s in enumerate(sl[:n.value])]

    def Contents(self) -> Dict[bytes, List[bytes]]:
        """key -> [value bytes of cpu 0 .. Indices()-1] (one bulk read per cpu)."""
        S = self.Spec.ValueSize
        ents = self.Entries()
        vals = [bytes(r) for r in self.ValuesRange(0, self.Indices())]
        return {k: [v[s * S:(s + 1) * S] for v in vals] for k, s in ents}

    def ValueOf(self, key: bytes, cpuid: int = 0) -> Optional[bytes]:
        """The value bytes for key on a cpu (Lookup + MemoryController read), None if absent."""
        a = self.Lookup(key, cpuid)
        return None if a == 0 else self._vm.MemoryController.Read(a, self.Spec.ValueSize)


class LinuxPerCPUHashMap(LinuxHashMap):  # emulator_linux_map_hash.go:417-664
    def Indices(self) -> int:
        return self._vm.settings.vcpus


HASH_TYPES = (1, 13, 18, 19, 24, 25, 26, 28, 29)
PERCPU_HASH_TYPES = (5, 21)


def MapSpecToLinuxMap(spec: MapSpec) -> LinuxMap:  # emulator_linux_map.go:57-113
    t = int(spec.Type)
    if t in (2, 3, 8, 12, 14, 15, 16, 17, 20):
        return LinuxArrayMap(spec)
    if t == 6:
        return LinuxPerCPUArrayMap(spec)
    if t in HASH_TYPES:
        return LinuxHashMap(spec)
    if t in PERCPU_HASH_TYPES:
        return LinuxPerCPUHashMap(spec)
    raise MimicError(f"unsupported map type '{t}' in this engine build")


# ---------------------------------------------------------------------------------------------
# contexts
# ---------------------------------------------------------------------------------------------

@dataclass
class LinuxContextXDP:  # context_xdp_md.go:22-34
    Headroom: int = 0
    Tailroom: int = 0
    Packet: bytes = b""
    IngessIfIndex: int = 0
    RxQueueIndex: int = 0
    EgressIfIndex: int = 0
    Name: str = ""


@dataclass
class NetDev:  # emulator_linux_sk_buff.go:962-964
    IFIndex: int = 0


def _jget(obj: dict, key: str, default=None):
    """encoding/json's field match: exact key first, then case-insensitive."""
    if key in obj:
        return obj[key]
    lk = key.lower()
    for k, v in obj.items():
        if k.lower() == lk:
            return v
    return default


def _parse_ip(text: str) -> Optional[bytes]:
    """net.ParseIP: 16 bytes for a valid IPv4 (::ffff:a.b.c.d) or IPv6 address, else None."""
    import ipaddress

    if not text or "%" in text:
        return None
    try:
        ip = ipaddress.ip_address(text)
    except ValueError:
        return None
    if ip.version == 4:
        return b"\x00" * 10 + b"\xff\xff" + ip.packed
    return ip.packed


@dataclass
class SK:  # emulator_linux_sk_buff.go:698-718 (JSON "sock" of an sk_buff context)
    """A user-given socket.  Its addresses are read through net.IP fields that only SK's
    UnmarshalJSON fills (:721-757): ``FromJSON`` sets them as it does (make(net.IP, 4 / 16), or the
    16 bytes of net.ParseIP); an SK made directly has nil addresses (reads panic), as a Go SK
    literal would."""
    BoundDevIF: int = 0
    Family: int = 0
    SockType: int = 0
    Protocol: int = 0
    Mark: int = 0
    Priority: int = 0
    SrcIP4: str = ""
    SrcIP6: str = ""
    SrcPort: int = 0
    DstPort: int = 0
    DstIP4: str = ""
    DstIP6: str = ""
    State: int = 0
    RXQueueMapping: int = 0
    ips: Optional[Tuple[bytes, bytes, bytes, bytes]] = None   # srcIP4, dstIP4, srcIP6, dstIP6 (None: nil)

    @classmethod
    def FromJSON(cls, obj: dict) -> "SK":
        u = lambda k: int(_jget(obj, k, 0) or 0) & 0xFFFFFFFF   # noqa: E731
        sk = cls(BoundDevIF=u("boundDevIF"), Family=u("family"), SockType=u("sockType"), Protocol=u("protocol"),
                 Mark=u("mark"), Priority=u("priority"), SrcIP4=_jget(obj, "srcIP4", "") or "",
                 SrcIP6=_jget(obj, "srcIP6", "") or "", SrcPort=u("srcPort"), DstPort=u("dstPort"),
                 DstIP4=_jget(obj, "dstIP4", "") or "", DstIP6=_jget(obj, "dstIP6", "") or "", State=u("state"),
                 RXQueueMapping=int(_jget(obj, "rxQueueMapping", 0) or 0))
        # UnmarshalJSON: make(net.IP, 4 / 16), replaced by net.ParseIP's bytes when it parses
        # (DstIP6 / SrcIP6 through To16, which keeps 16 bytes)
        sk.ips = tuple(_parse_ip(t) or bytes(n) for t, n in ((sk.SrcIP4, 4), (sk.DstIP4, 4), (sk.SrcIP6, 16),
                                                             (sk.DstIP6, 16)))
        return sk


@dataclass
class FlowKeys:  # emulator_linux_sk_buff.go:967-982 (JSON "flowKeys" of an sk_buff context)
    """User-given flow keys: the values the program's bpf_flow_keys start from.  SrcIPv6orIPv4 is
    kept for the JSON surface; no access reaches it (convertAccess panics at offsets 16..31)."""
    Nhoff: int = 0
    Thoff: int = 0
    AddrProto: int = 0
    IsFrag: int = 0
    IsFirstFrag: int = 0
    IsEncap: int = 0
    IPProto: int = 0
    NProto: int = 0
    Sport: int = 0
    Dport: int = 0
    SrcIPv6orIPv4: Optional[bytes] = None
    Flags: int = 0
    FlowLabel: int = 0

    @classmethod
    def FromJSON(cls, obj: dict) -> "FlowKeys":
        g = lambda k, m: int(_jget(obj, k, 0) or 0) & m   # noqa: E731
        ip = _jget(obj, "ip")
        return cls(Nhoff=g("nhoff", 0xFFFF), Thoff=g("thoff", 0xFFFF), AddrProto=g("addrProto", 0xFFFF),
                   IsFrag=g("isFrag", 0xFF), IsFirstFrag=g("isFirstFrag", 0xFF), IsEncap=g("isEncap", 0xFF),
                   IPProto=g("ipProto", 0xFF), NProto=g("nProto", 0xFFFF), Sport=g("sport", 0xFFFF),
                   Dport=g("dport", 0xFFFF), SrcIPv6orIPv4=_parse_ip(ip) if isinstance(ip, str) else None,
                   Flags=g("flags", 0xFFFFFFFF), FlowLabel=g("flowLabel", 0xFFFFFFFF))


@dataclass
class LinuxContextSKBuff:  # context_sk_buff.go:20-29
    """An sk_buff context: the packet, the device, and optionally a user-given socket / flow keys
    that Load puts in place of the ones SKBuffFromBytes derives (context_sk_buff.go:53-66)."""
    Packet: bytes = b""
    Dev: Optional[NetDev] = None
    Name: str = ""
    SK: Optional["SK"] = None
    FlowKeys: Optional["FlowKeys"] = None


def skb_custom_record(ctx: "LinuxContextSKBuff"):
    """The mimic_skb_custom entry (include/mimic_amd.h) of a context: a numpy record whose flags
    are 0 when the context gives neither a socket nor flow keys."""
    import numpy as np

    r = np.zeros((), L.SKB_CUSTOM_DTYPE)
    sk, fk = ctx.SK, ctx.FlowKeys
    if sk is not None:
        r["flags"] |= L.SKB_CUSTOM_SK
        for f, v in (("sk_bound_dev_if", sk.BoundDevIF), ("sk_family", sk.Family), ("sk_type", sk.SockType),
                     ("sk_protocol", sk.Protocol), ("sk_mark", sk.Mark), ("sk_priority", sk.Priority),
                     ("sk_src_port", sk.SrcPort), ("sk_dst_port", sk.DstPort), ("sk_state", sk.State)):
            r[f] = int(v) & 0xFFFFFFFF
        r["sk_rx_queue_mapping"] = int(sk.RXQueueMapping)
        for k, ip in enumerate(sk.ips or (None,) * 4):
            b = bytes(ip or b"")[:16]
            r["sk_ip_len"][k] = len(b)
            r["sk_ip"][k][:len(b)] = np.frombuffer(b, np.uint8)
    if fk is not None:
        r["flags"] |= L.SKB_CUSTOM_FLOWKEYS
        for f, v in (("fk_nhoff", fk.Nhoff), ("fk_thoff", fk.Thoff), ("fk_addr_proto", fk.AddrProto),
                     ("fk_is_frag", fk.IsFrag), ("fk_is_first_frag", fk.IsFirstFrag), ("fk_is_encap", fk.IsEncap),
                     ("fk_ip_proto", fk.IPProto), ("fk_n_proto", fk.NProto), ("fk_sport", fk.Sport),
                     ("fk_dport", fk.Dport), ("fk_flags", fk.Flags), ("fk_flow_label", fk.FlowLabel)):
            r[f] = v
    return r


def UnmarshalContextJSON(text: str):
    """context.go:57-71 + context_xdp_md.go:10-19 + context_sk_buff.go:8-17."""
    obj = json.loads(text)
    typ = obj.get("type")
    c = obj.get("ctx") or {}
    if typ == "sk_buff":
        pkt = c.get("packet")
        dev = c.get("dev")
        sock, fks = _jget(c, "sock"), _jget(c, "flowKeys")
        return LinuxContextSKBuff(Packet=base64.b64decode(pkt) if pkt else b"",
                                  Dev=NetDev(int(dev.get("ifIndex", 0))) if dev is not None else None,
                                  Name=obj.get("name", ""), SK=SK.FromJSON(sock) if sock is not None else None,
                                  FlowKeys=FlowKeys.FromJSON(fks) if fks is not None else None)
    if typ != "xdp_md":
        raise MimicError(f"no context unmarshaller registered for type '{typ}'")
    pkt = c.get("packet")
    return LinuxContextXDP(Headroom=int(c.get("headroom", 0)), Tailroom=int(c.get("tailroom", 0)),
                           Packet=base64.b64decode(pkt) if pkt else b"",
                           IngessIfIndex=int(c.get("ingress_ifidx", 0)), RxQueueIndex=int(c.get("rx_queue_idx", 0)),
                           EgressIfIndex=int(c.get("egress_ifidx", 0)), Name=obj.get("name", ""))


# ---------------------------------------------------------------------------------------------
# VM
# ---------------------------------------------------------------------------------------------

def VMOptEmulator(e: LinuxEmulator):
    return ("emulator", e)


def VMOptSetvCPUs(n: int):
    return ("vcpus", n)


def VMOptDevice(d: int):
    return ("device", d)


def VMOptExecMode(mode: str):
    """'jit' (per-program-set kernels, the default), 'interp' (the batch interpreter) or
    'default' (the MIMIC_EXEC environment variable decides)."""
    return ("exec", {"default": 0, "interp": 1, "jit": 2}[mode])


def VMOptSpread(mode: int):
    """Spread launches (mimic_set_spread): -1 the default policy, 0 never, 1 whenever the loaded
    programs allow it (every per-CPU access a fused counter increment)."""
    return ("spread", mode)


def VMOptShard(begin: int, count: int):
    """Execute only vCPUs [begin, begin+count) on this engine (multi-GPU sharding)."""
    return ("shard", (begin, count))


@dataclass
class VMSettings:
    vcpus: int
    stack_frame_size: int = 256
    stack_frame_count: int = 8
    device: int = 0
    vcpu_begin: int = 0
    vcpu_count: int = 0
    exec_mode: int = 0


class MemoryControllerView:
    """Host inspection of device-resident static memory (memory_controller.go:117-145 + VMMem)."""

    def __init__(self, vm: "VM"):
        self.vm = vm

    def Read(self, addr: int, n: int) -> bytes:
        buf = C.create_string_buffer(max(n, 1))
        _check(self.vm.h, self.vm.lib.mimic_mem_read(self.vm.h, addr, buf, n), "mem read")
        return buf.raw[:n]

    def Load(self, addr: int, size: int) -> int:
        v = C.c_uint64()
        _check(self.vm.h, self.vm.lib.mimic_mem_load(self.vm.h, addr, size, C.byref(v)), "mem load")
        return v.value


class VM:
    def __init__(self, emulator: LinuxEmulator, settings: VMSettings):
        if emulator is None:  # vm.go:73 calls SetVM on a nil emulator
            raise MimicError("NewVM requires an emulator (the reference panics without one)")
        self.lib = L.load()
        self.settings = settings
        s = L.VMSettings(settings.vcpus, settings.stack_frame_size, settings.stack_frame_count,
                         emulator.MaxTailCalls, settings.device, settings.vcpu_begin, settings.vcpu_count,
                         settings.exec_mode)
        h = C.c_void_p()
        rc = self.lib.mimic_vm_create(C.byref(s), C.byref(h))
        if rc != 0:
            raise MimicError(f"mimic_vm_create failed ({rc})")
        self.h = h
        self.emulator = emulator
        self.MemoryController = MemoryControllerView(self)
        self.programs: List[ProgramSpec] = []
        emulator.SetVM(self)

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.mimic_vm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # vm.go:98-139
    def AddProgram(self, prog: ProgramSpec) -> int:
        raw = bytes(prog.Instructions)
        if len(raw) % 8:
            raise MimicError("instruction stream is not a multiple of 8 bytes")
        relocs = []
        for slot, name in prog.References:
            m = self.emulator.Maps.get(name)
            if m is None:
                raise MimicError(f"program references a map named '{name}', no map with that name exists in the emulator")
            relocs.append(L.Reloc(slot, m.id))
        arr = (L.Reloc * max(len(relocs), 1))(*relocs)
        pid = C.c_uint32()
        buf = C.create_string_buffer(raw, max(len(raw), 1))
        _check(self.h, self.lib.mimic_program_load(self.h, prog.Name.encode(), buf, len(raw) // 8, arr, len(relocs),
                                                   C.byref(pid)), "AddProgram")
        self.programs.append(prog)
        return pid.value

    def GetProcessPool(self) -> "ProcessPool":  # vm.go:79-81
        if getattr(self, "_pool", None) is None:
            self._pool = ProcessPool(self)
        return self._pool

    def GetPrograms(self) -> List[ProgramSpec]:
        return list(self.programs)

    def ProgramAddress(self, prog_id: int) -> int:
        a = C.c_uint32()
        _check(self.h, self.lib.mimic_program_addr(self.h, prog_id, C.byref(a)), "program addr")
        return a.value

    def StackAddress(self) -> int:
        a = C.c_uint32()
        _check(self.h, self.lib.mimic_stack_addr(self.h, C.byref(a)), "stack addr")
        return a.value

    def NewProcess(self, entrypoint: int, ctx=None) -> "Process":  # vm.go:198-235
        if entrypoint >= len(self.programs):
            raise MimicError(f"no program with id '{entrypoint}' is loaded")
        return Process(self, entrypoint, ctx)

    # ---- batch entry point ------------------------------------------------------------------
    def RunXDPBatch(self, prog_id: int, batch: "XDPBatch", results: Optional["XDPResults"] = None,
                    stream=None, sync: bool = True, ctx: Optional["Context"] = None,
                    ctx_per_packet: Optional[Sequence[Optional["Context"]]] = None) -> "XDPResults":
        """N x {NewProcess, SetCPUID, Run(ctx), read R0, Cleanup} on the GPU.  ctx: one context
        for every process, or ctx_per_packet: one each (None entries: Background)."""
        if results is None:
            results = XDPResults.empty(batch.n, batch.pkt_data.device)
        b = batch._c()
        r = results._c()
        st = stream.cuda_stream if stream is not None else None
        h, arr, _keep = _ctx_args(ctx, ctx_per_packet, batch.n)
        if h is not None or arr is not None:
            rc = self.lib.mimic_run_xdp_ctx(self.h, prog_id, b, r, st, h, arr)
        else:
            rc = self.lib.mimic_run_xdp(self.h, prog_id, b, r, st)
        if rc:
            _check(self.h, rc, "RunXDPBatch")
        if sync:
            _check(self.h, self.lib.mimic_sync(self.h, st), "sync")
        else:   # the launch reads the batch until it ends: the results keep it (and the contexts) alive
            results._inflight = (batch, _keep)
        return results

    def RunXDPMany(self, prog_id: int, batches: Sequence["XDPBatch"], results: Optional[Sequence["XDPResults"]] = None,
                   stream=None, sync: bool = True) -> List["XDPResults"]:
        """Several device batches of one program (mimic_run_xdp_many): up to 8 of one shape run as ONE
        launch when the programs allow the owned spread kernel, each vCPU running its packets of
        batch 0, then batch 1, ... (a processPool draining a backlog, vm.go:548-573); else one launch
        per batch.  Not in the reference API."""
        if results is None:
            results = [XDPResults.empty(b.n, b.pkt_data.device) for b in batches]
        k = len(batches)
        bs, rs = (L.XDPBatch * max(k, 1))(), (L.XDPResults * max(k, 1))()
        for q, (bt, rt) in enumerate(zip(batches, results)):
            bt._c()
            rt._c()
            bs[q], rs[q] = bt._cstruct_obj, rt._cstruct_obj
        st = stream.cuda_stream if stream is not None else None
        rc = self.lib.mimic_run_xdp_many(self.h, prog_id, bs, rs, k, st)
        if rc:
            _check(self.h, rc, "RunXDPMany")
        if sync:
            _check(self.h, self.lib.mimic_sync(self.h, st), "sync")
        else:
            for bt, rt in zip(batches, results):
                rt._inflight = bt
        return list(results)

    def RunSKBBatch(self, prog_id: int, batch: "SKBBatch", results: Optional["XDPResults"] = None,
                    stream=None, sync: bool = True, ctx: Optional["Context"] = None,
                    ctx_per_packet: Optional[Sequence[Optional["Context"]]] = None) -> "XDPResults":
        """N x {NewProcess(LinuxContextSKBuff), SetCPUID, Run(ctx), read R0, Cleanup} on the GPU."""
        if results is None:
            results = XDPResults.empty(batch.n, batch.pkt_data.device)
        st = stream.cuda_stream if stream is not None else None
        h, arr, _keep = _ctx_args(ctx, ctx_per_packet, batch.n)
        if h is not None or arr is not None:
            rc = self.lib.mimic_run_skb_ctx(self.h, prog_id, batch._c(), results._c(), st, h, arr)
        else:
            rc = self.lib.mimic_run_skb(self.h, prog_id, batch._c(), results._c(), st)
        if rc:
            _check(self.h, rc, "RunSKBBatch")
        if sync:
            _check(self.h, self.lib.mimic_sync(self.h, st), "sync")
        else:
            results._inflight = (batch, _keep)
        return results

    def CleanupProcesses(self, procs: Sequence["Process"]) -> None:
        """Process.Cleanup of many processes (one wait for the VM's stream)."""
        nat = [p._native for p in procs if p._native is not None]
        if nat and getattr(self, "h", None):
            self.lib.mimic_process_free_many((C.c_void_p * len(nat))(*nat), len(nat))
        for p in procs:
            p._native = None

    def RunProcesses(self, procs: Sequence["Process"], ctxs: Optional[Sequence[Optional["Context"]]] = None,
                     cpus: Optional[Sequence[int]] = None) -> None:
        """processPool's workers for fresh sk_buff processes: Run(ctx) of every process as ONE device
        launch (mimic_process_run_many), each with the leak addresses its NewProcess reserved and on
        its SetCPUID vCPU.  Afterwards each process has R0, Status, Steps and ErrPC (registers R1-R10
        are not kept by a batch lane); a fatal status is left in Status (not raised)."""
        n = len(procs)
        if not n:
            return
        for p in procs:
            p._ensure_native()
        arr = (C.c_void_p * n)(*[p._native for p in procs])
        cx = None
        if ctxs is not None and any(_live(c) is not None for c in ctxs):
            hs = {}
            for c in ctxs:
                if _live(c) is not None and id(c) not in hs:
                    hs[id(c)] = c._device_handle()
            cx = (C.c_void_p * n)(*[hs[id(c)] if _live(c) is not None else None for c in ctxs])
        import numpy as np

        regs = (L.ProcessRegs * n)()
        ca = None
        if cpus is not None:
            ca = np.ascontiguousarray(cpus, dtype=np.int32)
        _check(self.h, self.lib.mimic_process_run_many(arr, n, ca.ctypes.data if ca is not None else None, cx, regs),
               "RunProcesses")
        a = np.ctypeslib.as_array(regs)   # one column per field, not a ctypes access per field
        r0, steps = a["r"][:, 0].tolist(), a["steps"].tolist()
        sts, pcs = a["status"].tolist(), a["pc"].tolist()
        for p, x, s, st, pc in zip(procs, r0, steps, sts, pcs):   # what a batch lane keeps: R0, status, steps
            p.Registers.R0 = x
            p.Steps = s
            p.Status = st
            p._exited = True
            p._started = True
            p.ErrPC = pc if st else -1

    def SKBRelease(self) -> None:
        """Forget the sock / flow-keys / packet entries earlier sk_buff processes leaked (a fresh
        VM with the same maps and programs)."""
        _check(self.h, self.lib.mimic_skb_release(self.h), "skb release")

    def RunXDPHost(self, prog_id: int, buf, off, lens, schedule=L.SCHED_INTERLEAVED, cpu=None, headroom: int = 0,
                   tailroom: int = 0, ingress: int = 0, rxq: int = 0, egress: int = 0, step_budget: int = 0,
                   chunks: int = 0, pkt_out=None, r0=None, status=None, ctx: Optional["Context"] = None,
                   ctx_per_packet: Optional[Sequence[Optional["Context"]]] = None):
        """A batch resident in HOST memory (numpy arrays): the engine pipelines H2D copies, the
        kernels and the D2H copies of r0/status (and of the packet memory into pkt_out).
        Returns (r0 uint64[n], status uint8[n]).  Register the arrays (HostRegister) for
        asynchronous copies.  Run(ctx): one context for the batch, or one per packet
        (ctx_per_packet, as processPool's jobs carry theirs)."""
        import numpy as np

        n = len(lens)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        r0 = np.empty(n, np.uint64) if r0 is None else r0
        status = np.empty(n, np.uint8) if status is None else status
        hb = L.XDPHostBatch()
        hb.n, hb.schedule = n, schedule
        hb.pkt_data, hb.pkt_off, hb.pkt_len = buf.ctypes.data, off.ctypes.data, lens.ctypes.data
        hb.headroom_all, hb.tailroom_all = headroom, tailroom
        hb.ingress_all, hb.rxq_all, hb.egress_all = ingress, rxq, egress
        cpu_arr = None
        if cpu is not None:
            cpu_arr = np.ascontiguousarray(cpu, dtype=np.int32)
            hb.cpu = cpu_arr.ctypes.data
        hb.step_budget = step_budget
        hb.pkt_out = pkt_out.ctypes.data if pkt_out is not None else None
        hb.r0, hb.status = r0.ctypes.data, status.ctypes.data
        h, arr, _keep = _ctx_args(ctx, ctx_per_packet, n)
        if h is not None:   # Run(ctx): every sub-batch's kernel reads the context
            _check(self.h, self.lib.mimic_run_xdp_host_ctx(self.h, prog_id, C.byref(hb), chunks, h), "RunXDPHost")
        elif arr is not None:   # one context per packet
            _check(self.h, self.lib.mimic_run_xdp_host_ctx_pp(self.h, prog_id, C.byref(hb), chunks, arr), "RunXDPHost")
        else:
            _check(self.h, self.lib.mimic_run_xdp_host(self.h, prog_id, C.byref(hb), chunks), "RunXDPHost")
        return r0, status

    def HostRegister(self, arr) -> None:
        """Pin a numpy array's memory for DMA (hipHostRegister)."""
        _check(self.h, self.lib.mimic_host_register(arr.ctypes.data, arr.nbytes), "host register")

    def HostUnregister(self, arr) -> None:
        _check(self.h, self.lib.mimic_host_unregister(arr.ctypes.data), "host unregister")

    def LastSteps(self) -> int:
        v = C.c_uint64()
        _check(self.h, self.lib.mimic_last_steps(self.h, C.byref(v)), "last steps")
        return v.value

    def ExecMode(self) -> str:
        """'jit' (per-program-set kernels, hipRTC) or 'interp' (the batch interpreter)."""
        return {1: "interp", 2: "jit"}[self.lib.mimic_exec_mode(self.h)]

    def LastExec(self) -> str:
        """The kernel the last batch ran on."""
        return {0: "none", 1: "interp", 2: "jit", 3: "spread", 4: "spread_own"}[self.lib.mimic_last_exec(self.h)]

    def SetSpread(self, mode: int) -> None:
        """Spread launches (mimic_set_spread): -1 default policy, 0 never, 1 whenever allowed."""
        _check(self.h, self.lib.mimic_set_spread(self.h, mode), "SetSpread")


def NewVM(*opts) -> VM:  # vm.go:54-76
    emu = None
    spread = None
    s = VMSettings(vcpus=os.cpu_count() or 1)  # VirtualCPUs defaults to runtime.NumCPU()
    for k, v in opts:
        if k == "emulator":
            emu = v
        elif k == "vcpus":
            s.vcpus = v
        elif k == "device":
            s.device = v
        elif k == "shard":
            s.vcpu_begin, s.vcpu_count = v
        elif k == "exec":
            s.exec_mode = v
        elif k == "spread":
            spread = v
    vm = VM(emu, s)
    if spread is not None:
        vm.SetSpread(spread)
    return vm


class Registers:
    """Process.Registers (vm.go:378-405): PC and R0..R10."""

    def __init__(self):
        self.PC = 0
        for q in range(11):
            setattr(self, f"R{q}", 0)

    def Get(self, r: int) -> int:
        return getattr(self, f"R{r}")


class Process:
    """A process of the VM (vm.go:238-374), held on the device (mimic_process_*): Step()
    advances it one instruction at a time (a single-lane interpreter launch per call), Run()
    runs it to the end (continuing a stepped process), and every register is readable after
    either.  An sk_buff process's context Load runs at NewProcess, as in the reference
    (context_sk_buff.go:42-107: its leaked entries take the VM's next addresses then).  Batches
    of processes run through VM.RunXDPBatch / RunSKBBatch instead."""

    def __init__(self, vm: VM, prog_id: int, ctx=None):
        self.VM = vm
        self.prog_id = prog_id
        self.Context = ctx
        self.Registers = Registers()
        self.cpuID = -1
        self.Steps = 0
        self.Status = None
        self.ErrPC = -1
        self.PacketAfter: Optional[bytes] = None
        self._native = None
        self._exited = False
        self._started = False   # stepped or run at least once
        self.Registers.R10 = vm.StackAddress() + vm.settings.stack_frame_size   # vm.go:224
        if isinstance(ctx, LinuxContextSKBuff):
            self._ensure_native()

    def CPUID(self) -> int:
        return self.cpuID

    def SetCPUID(self, i: int) -> None:  # vm.go:268-283
        if i < 0:
            raise MimicError("not a valid CPU ID")
        if i > self.VM.settings.vcpus:
            raise MimicError(f"vm only has {self.VM.settings.vcpus} vCPUs, max CPU ID is {self.VM.settings.vcpus - 1}")
        self.cpuID = i
        if self._native is not None:
            _check(self.VM.h, self.VM.lib.mimic_process_set_cpu(self._native, i), "SetCPUID")

    # ---- stepping (device-resident single process) -----------------------------------------
    def _ensure_native(self):
        if self._native is not None:
            return
        ctx = self.Context or LinuxContextXDP()
        h = C.c_void_p()
        pkt = bytes(ctx.Packet)
        if isinstance(ctx, LinuxContextSKBuff):   # its Load (leak addresses) happens here, as in NewProcess
            cust = skb_custom_record(ctx)
            cp = cust.ctypes.data if int(cust["flags"]) else None
            _check(self.VM.h, self.VM.lib.mimic_process_new_skb_ctx(self.VM.h, self.prog_id, pkt, len(pkt),
                                                                     ctx.Dev.IFIndex if ctx.Dev else 0, cp, C.byref(h)),
                   "NewProcess")
        else:
            _check(self.VM.h, self.VM.lib.mimic_process_new(self.VM.h, self.prog_id, pkt, len(pkt), ctx.Headroom,
                                                             ctx.Tailroom, ctx.IngessIfIndex, ctx.RxQueueIndex,
                                                             ctx.EgressIfIndex, C.byref(h)), "NewProcess")
        self._native = h
        if self.cpuID >= 0:
            _check(self.VM.h, self.VM.lib.mimic_process_set_cpu(h, self.cpuID), "SetCPUID")

    def _take(self, regs) -> None:
        for q in range(11):
            setattr(self.Registers, f"R{q}", int(regs.r[q]))
        self.Registers.PC = int(regs.pc)
        self.ProgramID = int(regs.prog_id)
        self.Steps = int(regs.steps)
        self.Status = int(regs.status)
        self._exited = bool(regs.exited)

    def Step(self) -> bool:
        """Process.Step (vm.go:291-340): execute one instruction; True once the program exited.
        A fatal error raises MimicError (the reference returns it), after which the process is
        terminated."""
        self._ensure_native()
        self._started = True
        regs = L.ProcessRegs()
        rc = self.VM.lib.mimic_process_step(self._native, 1, C.byref(regs))
        if rc < 0:
            _check(self.VM.h, rc, "Step")
        self._take(regs)
        if self.Status:
            self.ErrPC = self.Registers.PC
            raise MimicError(f"inst at PC({self.Registers.PC}): {L.STATUS_NAMES[self.Status]}")
        return self._exited

    def Run(self, step_budget: int = 0, ctx: Optional["Context"] = None) -> None:  # vm.go:343-360
        """Process.Run: run to exit (or a fatal error, or the step budget standing in for the
        context deadline).  Every register is readable afterwards (Registers.R0..R10, PC), as
        after the reference's Run (Readme.md:74-78): the process runs on the device as a
        single-lane launch that saves its whole state (mimic_process_run), continuing a process
        that Step() has started.  cpuID stays -1 when SetCPUID was never called (vm.go:214) and may
        equal V (vm.go:273): the reference runs such processes; only per-CPU map operations fail
        in them (emulator_linux_map_array.go:236-238).  With ctx, Run(ctx): the context is checked
        between launch slices; once it is done Run raises MimicError(ctx.Err()) with the process
        suspended (Run / Step continue it), and step_budget 0 means no step budget."""
        self._ensure_native()
        self._started = True
        regs = L.ProcessRegs()
        if ctx is not None:
            rc = self.VM.lib.mimic_process_run_ctx(self._native, step_budget, ctx._device_handle(), C.byref(regs))
            if rc in (L.ECANCELED, L.EDEADLINE):
                self._take(regs)
                raise MimicError(Context._ERR[1 if rc == L.ECANCELED else 2])
            _check(self.VM.h, rc, "Run")
        else:
            _check(self.VM.h, self.VM.lib.mimic_process_run(self._native, step_budget, C.byref(regs)), "Run")
        self._take(regs)
        self.ErrPC = self.Registers.PC if self.Status else -1
        self.PacketAfter = self.Packet()
        if self.Status:
            raise MimicError(f"process encountered a fatal error: {L.STATUS_NAMES[self.Status]} at PC({self.ErrPC})")

    def Packet(self) -> bytes:
        """Packet memory (headroom + packet + tailroom) of a stepped process, as it is now."""
        if self._native is None:
            return self.PacketAfter or b""
        ctx = self.Context or LinuxContextXDP()
        if isinstance(ctx, LinuxContextSKBuff):
            n = 32 + len(ctx.Packet) + 64   # emulator_linux_sk_buff.go:113-116
        else:
            n = ctx.Headroom + len(ctx.Packet) + ctx.Tailroom
        buf = C.create_string_buffer(max(n, 1))
        _check(self.VM.h, self.VM.lib.mimic_process_packet(self._native, buf, max(n, 1)), "packet")
        return buf.raw[:n]

    def Cleanup(self) -> None:  # vm.go:363-374
        if self._native is not None and getattr(self.VM, "h", None):   # (a closed VM freed its device state)
            self.VM.lib.mimic_process_free(self._native)
        self._native = None

    def __del__(self):
        try:
            self.Cleanup()
        except Exception:
            pass


# ---------------------------------------------------------------------------------------------
# batch containers (device tensors)
# ---------------------------------------------------------------------------------------------

class XDPBatch:
    """A batch of xdp_md contexts resident on the GPU (see mimic_xdp_batch)."""

    def __init__(self, pkt_data, pkt_off, pkt_len, headroom=0, tailroom=0, ingress=0, rxq=0, egress=0,
                 schedule=L.SCHED_CHUNKED, cpu=None, step_budget=0):
        self.pkt_data, self.pkt_off, self.pkt_len = pkt_data, pkt_off, pkt_len
        self.headroom, self.tailroom = headroom, tailroom
        self.ingress, self.rxq, self.egress = ingress, rxq, egress
        self.schedule, self.cpu, self.step_budget = schedule, cpu, step_budget

    @property
    def n(self) -> int:
        return int(self.pkt_len.numel())

    def _c(self):
        """The mimic_xdp_batch of this batch (built once; a batch is not modified after use)."""
        cached = getattr(self, "_cstruct", None)
        if cached is not None:
            return cached
        import torch

        b = L.XDPBatch()
        b.n = self.n
        b.schedule = self.schedule
        b.pkt_data = self.pkt_data.data_ptr()
        b.pkt_off = self.pkt_off.data_ptr()
        b.pkt_len = self.pkt_len.data_ptr()
        b.headroom = self.headroom.data_ptr() if isinstance(self.headroom, torch.Tensor) else None
        b.headroom_all = 0 if isinstance(self.headroom, torch.Tensor) else int(self.headroom)
        b.tailroom = self.tailroom.data_ptr() if isinstance(self.tailroom, torch.Tensor) else None
        b.tailroom_all = 0 if isinstance(self.tailroom, torch.Tensor) else int(self.tailroom)
        for fld, allname, val in (("ingress_ifindex", "ingress_all", self.ingress), ("rx_queue_index", "rxq_all", self.rxq),
                                  ("egress_ifindex", "egress_all", self.egress)):
            if isinstance(val, torch.Tensor):
                setattr(b, fld, val.data_ptr())
                setattr(b, allname, 0)
            else:
                setattr(b, fld, None)
                setattr(b, allname, int(val))
        self._cpu_host = None
        if self.schedule == L.SCHED_EXPLICIT:
            import numpy as np

            self._cpu_host = np.ascontiguousarray(np.asarray(self.cpu, dtype=np.int32))
            b.cpu = self._cpu_host.ctypes.data
        else:
            b.cpu = None
        b.step_budget = self.step_budget
        self._cstruct = C.byref(b)
        self._cstruct_obj = b
        return self._cstruct

    @staticmethod
    def layout(lengths: Sequence[int], headroom=0, tailroom=0, align: int = 64):
        """Offsets of each packet memory (H+L+T) in one buffer, each aligned to `align`."""
        import numpy as np

        lens = np.asarray(lengths, dtype=np.int64)
        H = np.asarray(headroom, dtype=np.int64) if not np.isscalar(headroom) else np.full(lens.shape, headroom)
        T = np.asarray(tailroom, dtype=np.int64) if not np.isscalar(tailroom) else np.full(lens.shape, tailroom)
        sizes = (H + lens + T + align - 1) // align * align
        off = np.zeros(lens.shape, dtype=np.int64)
        if len(lens) > 1:
            off[1:] = np.cumsum(sizes)[:-1]
        total = int(sizes.sum()) if len(lens) else 0
        return off.astype(np.uint64), total

    @classmethod
    def from_packets(cls, packets: Sequence[bytes], device="cuda", headroom=0, tailroom=0, ingress=0, rxq=0,
                     egress=0, schedule=L.SCHED_CHUNKED, cpu=None, step_budget=0):
        import numpy as np
        import torch

        lens = [len(p) for p in packets]
        H_arr = None if np.isscalar(headroom) else np.asarray(headroom, dtype=np.uint32)
        T_arr = None if np.isscalar(tailroom) else np.asarray(tailroom, dtype=np.uint32)
        off, total = cls.layout(lens, headroom, tailroom)
        buf = np.zeros(max(total, 1), dtype=np.uint8)
        for i, p in enumerate(packets):
            h = int(H_arr[i]) if H_arr is not None else int(headroom)
            buf[int(off[i]) + h:int(off[i]) + h + len(p)] = np.frombuffer(bytes(p), dtype=np.uint8)
        return cls.from_numpy(buf, off, np.asarray(lens, dtype=np.uint32), device, H_arr if H_arr is not None
                              else headroom, T_arr if T_arr is not None else tailroom, ingress, rxq, egress,
                              schedule, cpu, step_budget)

    @classmethod
    def from_numpy(cls, buf, off, lens, device="cuda", headroom=0, tailroom=0, ingress=0, rxq=0, egress=0,
                   schedule=L.SCHED_CHUNKED, cpu=None, step_budget=0):
        import numpy as np
        import torch

        def t(a, dt):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=dt))).to(device)

        def opt(v, dt):
            return v if np.isscalar(v) else t(v, dt)

        return cls(t(buf, np.uint8), t(np.asarray(off, dtype=np.uint64).view(np.int64), np.int64),
                   t(np.asarray(lens, dtype=np.uint32).view(np.int32), np.int32),
                   opt(headroom, np.int32), opt(tailroom, np.int32), opt(ingress, np.int32), opt(rxq, np.int32),
                   opt(egress, np.int32), schedule, cpu, step_budget)

    def packet_bytes(self, i: int) -> bytes:
        """Packet memory i (H+L+T bytes) as it is now on the device."""
        import numpy as np

        o = int(self.pkt_off[i].item())
        h = int(self.headroom[i].item()) if not np.isscalar(self.headroom) else int(self.headroom)
        t_ = int(self.tailroom[i].item()) if not np.isscalar(self.tailroom) else int(self.tailroom)
        n = h + int(self.pkt_len[i].item()) + t_
        return bytes(self.pkt_data[o:o + n].cpu().numpy().tobytes())


class SKBBatch:
    """A batch of sk_buff contexts resident on the GPU (see mimic_skb_batch): packet memory i is
    32 + L + 64 bytes at pkt_off[i], the packet at +32."""
    HEADROOM, TAILROOM = 32, 64

    def __init__(self, pkt_data, pkt_off, pkt_len, ifindex=0, schedule=L.SCHED_CHUNKED, cpu=None, step_budget=0,
                 custom=None):
        self.pkt_data, self.pkt_off, self.pkt_len = pkt_data, pkt_off, pkt_len
        self.ifindex, self.schedule, self.cpu, self.step_budget = ifindex, schedule, cpu, step_budget
        self.custom = custom   # device uint8 tensor [n * sizeof(mimic_skb_custom)] or None

    @property
    def n(self) -> int:
        return int(self.pkt_len.numel())

    def _c(self):
        cached = getattr(self, "_cstruct", None)
        if cached is not None:
            return cached
        b = L.SKBBatch()
        b.n, b.schedule = self.n, self.schedule
        b.pkt_data, b.pkt_off, b.pkt_len = self.pkt_data.data_ptr(), self.pkt_off.data_ptr(), self.pkt_len.data_ptr()
        b.ifindex = int(self.ifindex)
        self._cpu_host = None
        if self.schedule == L.SCHED_EXPLICIT:
            import numpy as np

            self._cpu_host = np.ascontiguousarray(np.asarray(self.cpu, dtype=np.int32))
            b.cpu = self._cpu_host.ctypes.data
        else:
            b.cpu = None
        b.step_budget = self.step_budget
        b.custom = self.custom.data_ptr() if self.custom is not None else None
        if getattr(self, "rooms_state", None) is None:
            import torch

            # the engine's rooms-clean word for this batch's packets (mimic_skb_batch.rooms_state)
            self.rooms_state = torch.zeros(1, dtype=torch.int32, device=self.pkt_data.device)
        b.rooms_state = self.rooms_state.data_ptr()
        self._cstruct_obj = b
        self._cstruct = C.byref(b)
        return self._cstruct

    def PacketsWritten(self) -> None:
        """The packet memory was written by other means than the engine's runs: the next run reads
        every room again (mimic_skb_batch.rooms_state)."""
        if getattr(self, "rooms_state", None) is not None:
            self.rooms_state.zero_()

    @classmethod
    def layout(cls, lengths: Sequence[int], align: int = 64):
        return XDPBatch.layout(lengths, cls.HEADROOM, cls.TAILROOM, align)

    @staticmethod
    def custom_array(contexts: Sequence["LinuxContextSKBuff"]):
        """The mimic_skb_custom table (numpy) of a batch's contexts, or None when none gives a
        socket or flow keys."""
        import numpy as np

        recs = np.zeros(len(contexts), L.SKB_CUSTOM_DTYPE)
        for i, c in enumerate(contexts):
            recs[i] = skb_custom_record(c)
        return recs if recs["flags"].any() else None

    @classmethod
    def from_packets(cls, packets: Sequence[bytes], device="cuda", ifindex=0, schedule=L.SCHED_CHUNKED, cpu=None,
                     step_budget=0, custom=None):
        import numpy as np

        lens = np.asarray([len(p) for p in packets], dtype=np.uint32)
        off, total = cls.layout(lens)
        buf = np.zeros(max(total, 1), dtype=np.uint8)
        for i, p in enumerate(packets):
            o = int(off[i]) + cls.HEADROOM
            buf[o:o + len(p)] = np.frombuffer(bytes(p), dtype=np.uint8)
        return cls.from_numpy(buf, off, lens, device, ifindex, schedule, cpu, step_budget, custom)

    @classmethod
    def from_numpy(cls, buf, off, lens, device="cuda", ifindex=0, schedule=L.SCHED_CHUNKED, cpu=None, step_budget=0,
                   custom=None):
        """custom: a numpy mimic_skb_custom table (custom_array / skb_custom_record), one entry per
        packet, or None."""
        import numpy as np
        import torch

        def t(a, dt):
            return torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=dt))).to(device)

        cu = None
        if custom is not None:
            ca = np.ascontiguousarray(custom)
            if ca.dtype != L.SKB_CUSTOM_DTYPE or len(ca) != len(lens):
                raise MimicError("custom: one mimic_skb_custom entry per packet")
            cu = t(ca.view(np.uint8).reshape(-1), np.uint8)
        return cls(t(buf, np.uint8), t(np.asarray(off, dtype=np.uint64).view(np.int64), np.int64),
                   t(np.asarray(lens, dtype=np.uint32).view(np.int32), np.int32), ifindex, schedule, cpu, step_budget,
                   cu)

    def packet_bytes(self, i: int) -> bytes:
        o = int(self.pkt_off[i].item())
        n = self.HEADROOM + int(self.pkt_len[i].item()) + self.TAILROOM
        return bytes(self.pkt_data[o:o + n].cpu().numpy().tobytes())


class XDPResults:
    def __init__(self, r0, status, steps, err_pc):
        self.r0, self.status, self.steps, self.err_pc = r0, status, steps, err_pc

    def _c(self):
        cached = getattr(self, "_cstruct", None)
        if cached is None:
            def ptr(t):
                return t.data_ptr() if t is not None else None

            self._cstruct_obj = L.XDPResults(ptr(self.r0), ptr(self.status), ptr(self.steps), ptr(self.err_pc))
            cached = self._cstruct = C.byref(self._cstruct_obj)
        return cached

    @classmethod
    def empty(cls, n: int, device, full: bool = True):
        """full=False allocates only r0 and status (the process's R0 and error)."""
        import torch

        return cls(torch.zeros(max(n, 1), dtype=torch.int64, device=device),
                   torch.zeros(max(n, 1), dtype=torch.uint8, device=device),
                   torch.zeros(max(n, 1), dtype=torch.int32, device=device) if full else None,
                   torch.zeros(max(n, 1), dtype=torch.int32, device=device) if full else None)

    def numpy(self, n: Optional[int] = None):
        import numpy as np

        n = self.r0.numel() if n is None else n
        return {"r0": self.r0[:n].cpu().numpy().view(np.uint64), "status": self.status[:n].cpu().numpy(),
                "steps": self.steps[:n].cpu().numpy().view(np.uint32), "err_pc": self.err_pc[:n].cpu().numpy()}


# ---------------------------------------------------------------------------------------------
# ProcessPool (vm.go:468-583) on the device
# ---------------------------------------------------------------------------------------------
class Context:
    """context.Context as Run uses it (vm.go:343-360): Done / Err, made by Background(),
    WithCancel() or WithTimeout().  Deadline is a time.monotonic() value.  A context given to a
    device run is backed by a mimic_ctx (include/mimic_amd.h): a word in pinned host memory that the
    kernels read before each process's first step, set by Cancel() or by a native timer at the
    deadline, so a batch already running on the GPU stops starting processes once it is done."""

    _ERR = {1: "context canceled", 2: "context deadline exceeded"}

    def __init__(self, Deadline: Optional[float] = None, Cancelled: bool = False, _background: bool = False):
        self.Deadline = Deadline
        self.Cancelled = Cancelled
        self._background = _background   # context.Background(): never done, nothing to check
        self._h = None
        self._lib = None

    def Cancel(self) -> None:
        """The context's CancelFunc (context.Background() has none)."""
        if self._background:
            raise MimicError("context.Background() cannot be canceled")
        self.Cancelled = True
        if self._h is not None:
            self._lib.mimic_ctx_cancel(self._h)

    def _state(self) -> int:
        import time

        if self._h is not None:
            d = self._lib.mimic_ctx_err(self._h)
            if d:
                return d
        if self.Cancelled:
            return 1
        if self.Deadline is not None and time.monotonic() >= self.Deadline:
            return 2
        return 0

    def Err(self) -> Optional[str]:
        return self._ERR.get(self._state())

    def Done(self) -> bool:
        return self._state() != 0

    def native(self):
        """The mimic_ctx handle (made on first use; its state follows this context's)."""
        import time

        if self._h is None:
            lib = L.load()
            h = C.c_void_p()
            ns = 0
            if self.Deadline is not None:
                ns = max(1, int((self.Deadline - time.monotonic()) * 1e9))
            rc = lib.mimic_ctx_new(ns, C.byref(h))
            if rc:
                raise MimicError(f"context: error {rc}")
            self._lib, self._h = lib, h
            if self.Cancelled:   # (a passed deadline: the timer, armed at 1 ns, marks it)
                lib.mimic_ctx_cancel(h)
        return self._h

    def _device_handle(self):
        """The handle for a device run: the state so far carried over (a deadline already passed
        marks the word too)."""
        h = self.native()
        if not self._lib.mimic_ctx_err(h) and self._state() == 2 and self.Deadline is not None:
            # the deadline passed before the handle existed: the native timer (1 ns) marks it
            import time

            t_end = time.monotonic() + 1.0
            while not self._lib.mimic_ctx_err(h) and time.monotonic() < t_end:
                time.sleep(0)
        return h

    def close(self) -> None:
        if self._h is not None:
            self._lib.mimic_ctx_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def Background() -> Context:
    """context.Background(): never done.  A run given it takes the plain entry points (no pinned
    word, no context-checking kernel variant, spread launches allowed), as if no context were given."""
    return Context(_background=True)


def _live(ctx: Optional[Context]) -> Optional[Context]:
    """ctx, or None for context.Background() (which no kernel needs to read)."""
    return None if ctx is None or ctx._background else ctx


def WithCancel() -> Context:
    """context.WithCancel(context.Background()): done once Cancel() is called."""
    return Context()


def WithTimeout(seconds: float) -> Context:
    """context.WithTimeout(context.Background(), seconds)."""
    import time

    return Context(Deadline=time.monotonic() + seconds)


def _ctx_args(ctx, ctx_per_packet, n):
    """(handle, per-packet array, keep-alive) of a run's contexts."""
    if ctx is not None and ctx_per_packet is not None:
        raise MimicError("one context for the batch or one per packet, not both")
    ctx = _live(ctx)
    if ctx_per_packet is not None:
        if len(ctx_per_packet) != n:
            raise MimicError("one context per packet")
        ctx_per_packet = [_live(c) for c in ctx_per_packet]
        if all(c is None for c in ctx_per_packet):
            ctx_per_packet = None
    if ctx is not None:
        return ctx._device_handle(), None, None
    if ctx_per_packet is not None:
        if len(ctx_per_packet) != n:
            raise MimicError("one context per packet")
        hs = {}   # one handle per distinct context (a pool's jobs often share one)
        for c in ctx_per_packet:
            if c is not None and id(c) not in hs:
                hs[id(c)] = c._device_handle()
        arr = (C.c_void_p * n)(*[hs[id(c)] if c is not None else None for c in ctx_per_packet])
        return None, arr, arr
    return None, None, None


@dataclass
class ProcessPoolJob:  # vm.go:485-496
    Process: "Process"
    Context: Optional[Context] = None
    Handoff: Optional[object] = None   # callable(process, err: Optional[Exception])


class ProcessPool:
    """processPool (vm.go:468-583) the GPU way.  The reference runs V worker goroutines, worker c
    being vCPU c, each taking the next job off one channel and running it to completion.  Here one
    dispatcher thread drains the backlog in micro-batches: it gives the jobs vCPUs round-robin (a
    vCPU's jobs keep their enqueue order, so per-CPU map state is touched in order, the property
    the reference's pool guarantees) and runs each batch as ONE device launch with the EXPLICIT
    schedule -- thousands of vCPUs' processes at once instead of V goroutines.  Handoff callbacks
    run on their own threads (the reference starts a goroutine per handoff); without one the
    process is cleaned up."""

    def __init__(self, vm: VM, max_batch: int = 1 << 16):
        self.vm = vm
        self.max_batch = max_batch
        self._q = None
        self._thread = None
        self._next_cpu = 0

    def Start(self, backlog: int) -> None:
        import queue
        import threading

        if self._thread is not None:
            raise MimicError("pool is already running")
        if backlog < 1:
            raise MimicError("backlog must be at least 1")
        self._q = queue.Queue(maxsize=backlog)
        self._thread = threading.Thread(target=self._dispatch, name="mimic-process-pool", daemon=True)
        self._thread.start()

    def Enqueue(self, job: ProcessPoolJob, noblock: bool = False) -> None:
        import queue

        if self._thread is None:
            raise MimicError("pool is not yet running")
        if noblock:
            try:
                self._q.put_nowait(job)
            except queue.Full:
                raise MimicError("backlog is full") from None
        else:
            self._q.put(job)

    def Stop(self) -> None:
        """All pending jobs complete; returns when the dispatcher has exited."""
        if self._thread is None:
            return
        self._q.put(None)
        self._thread.join()
        self._thread = None
        self._q = None

    # ---- dispatcher ---------------------------------------------------------------------------
    def _handoff(self, job: ProcessPoolJob, err: Optional[Exception]) -> None:
        import threading

        if job.Handoff is not None:
            threading.Thread(target=job.Handoff, args=(job.Process, err), daemon=True).start()
        else:
            job.Process.Cleanup()

    def _dispatch(self) -> None:
        import queue

        done = False
        while not done:
            first = self._q.get()
            if first is None:
                break
            jobs = [first]
            while len(jobs) < self.max_batch:
                try:
                    j = self._q.get_nowait()
                except queue.Empty:
                    break
                if j is None:
                    done = True
                    break
                jobs.append(j)
            self._run(jobs)

    def _run(self, jobs) -> None:
        """One micro-batch: vCPUs round-robin, one launch per (program, context kind).  A vCPU runs
        its jobs in enqueue order (a worker takes them from the channel in order, vm.go:548-573):
        when the round-robin counter wraps inside the batch and a vCPU would get a job of a second
        group, the jobs so far run first."""
        V = self.vm.settings.vcpus
        groups: Dict[Tuple[int, bool, int], list] = {}
        owner: Dict[int, Tuple[int, bool, int]] = {}   # vCPU -> the group its jobs of this segment are in
        for job in jobs:
            err = job.Context.Err() if job.Context is not None else None
            if err is not None:
                self._handoff(job, MimicError(err))
                continue
            cpu = self._next_cpu
            skb = isinstance(job.Process.Context, LinuxContextSKBuff)
            # (sk_buff launches run one interface each: __sk_buff.ifindex is a launch parameter)
            ifx = (job.Process.Context.Dev.IFIndex if job.Process.Context.Dev else 0) if skb else 0
            key = (job.Process.prog_id, skb, ifx)
            if owner.get(cpu, key) != key:
                self._run_groups(groups)
                groups, owner = {}, {}
            if skb and not job.Process._started:
                job.Process.cpuID = cpu   # its native SetCPUID goes with the launch (RunProcesses cpus)
            else:
                job.Process.SetCPUID(cpu)
            self._next_cpu = (cpu + 1) % V
            owner[cpu] = key
            groups.setdefault(key, []).append(job)
        self._run_groups(groups)

    def _run_groups(self, groups) -> None:
        for (pid, skb, _ifx), js in groups.items():
            try:
                self._launch(pid, skb, js)
            except MimicError as ex:
                for job in js:
                    self._handoff(job, ex)
                continue
            done = []   # jobs without a handoff: cleaned up together (one stream wait)
            for job in js:
                p = job.Process
                err = None
                if p.Status in (L.STATUS["ERR_CANCELED"], L.STATUS["ERR_DEADLINE"]):   # Run returned ctx.Err()
                    err = MimicError(Context._ERR[p.Status - L.STATUS["ERR_CANCELED"] + 1])
                elif p.Status:
                    err = MimicError(f"process encountered a fatal error: {L.STATUS_NAMES[p.Status]} at PC({p.ErrPC})")
                if job.Handoff is None:
                    done.append(p)
                else:
                    self._handoff(job, err)
            self.vm.CleanupProcesses(done)

    def _launch(self, pid: int, skb: bool, js) -> None:
        dev = f"cuda:{self.vm.settings.device}"
        ctxs = [j.Process.Context or LinuxContextXDP() for j in js]
        cpus = [j.Process.cpuID for j in js]
        if skb:
            # An sk_buff process ran its context Load at NewProcess (its sock / flow keys / packet
            # took the VM's next leak addresses then, context_sk_buff.go:110-119), and the pool
            # worker only calls Run (vm.go:570).  The fresh processes of the group run as ONE launch
            # on the device processes NewProcess made, each with the addresses its Load reserved
            # (mimic_process_run_many); one a caller already stepped continues on its own.
            # (the group's jobs keep their order: fresh runs before a started job go first)
            fresh = []
            for j in js + [None]:
                if j is not None and not j.Process._started:
                    fresh.append(j)
                    continue
                if fresh:
                    self.vm.RunProcesses([f.Process for f in fresh], [f.Context for f in fresh],
                                         [f.Process.cpuID for f in fresh])
                    fresh = []
                if j is None:
                    break
                try:
                    j.Process.Run(ctx=j.Context)
                except MimicError as ex:
                    if str(ex) in Context._ERR.values():   # Run(ctx) returned ctx.Err()
                        j.Process.Status = L.STATUS["ERR_CANCELED"] + (str(ex) == Context._ERR[2])
                    elif not j.Process.Status:   # not a fatal status of the program: an engine error
                        raise
            return
        import numpy as np

        hr = [c.Headroom for c in ctxs]
        batch = XDPBatch.from_packets([c.Packet for c in ctxs], device=dev, headroom=np.array(hr, np.uint32),
                                      tailroom=np.array([c.Tailroom for c in ctxs], np.uint32),
                                      ingress=np.array([c.IngessIfIndex for c in ctxs], np.int32),
                                      rxq=np.array([c.RxQueueIndex for c in ctxs], np.int32),
                                      egress=np.array([c.EgressIfIndex for c in ctxs], np.int32),
                                      schedule=L.SCHED_EXPLICIT, cpu=cpus)
        # each job's context is checked on the device before its process's first step, so jobs
        # whose context is done while the launch runs stop there (vm.go:548-573)
        cpp = [j.Context for j in js] if any(j.Context is not None for j in js) else None
        res = self.vm.RunXDPBatch(pid, batch, ctx_per_packet=cpp).numpy(len(js))
        mem = batch.pkt_data.cpu().numpy()
        offs = batch.pkt_off.cpu().numpy()
        for k, j in enumerate(js):
            p = j.Process
            p.Registers.R0 = int(res["r0"][k]) & 0xFFFFFFFFFFFFFFFF
            p.Steps = int(res["steps"][k])
            p.Status = int(res["status"][k])
            p.ErrPC = int(res["err_pc"][k])
            c = ctxs[k]
            tail = c.Tailroom
            o = int(offs[k])
            p.PacketAfter = bytes(mem[o:o + hr[k] + len(c.Packet) + tail].tobytes())
