"""mimic_amd -- MI355X-native batch eBPF engine behind dylandreimerink/mimic's Process.Run surface.

Product path: per-program gfx950 JIT kernels (csrc/jit.cpp, hipRTC) and the hand-written batch
interpreter (csrc/interp.hip) + C++ host engine (csrc/engine.cpp) behind the C ABI in include/mimic_amd.h, bound here with ctypes.
"""
from .vm import (Background, Context, WithCancel, WithTimeout, ProcessPool, ProcessPoolJob, E2BIG, LinuxArrayMap, LinuxContextSKBuff, LinuxContextXDP, NetDev, SKBBatch, SK, FlowKeys, LinuxEmulator, LinuxHashMap, LinuxMap, LinuxPerCPUArrayMap,
                 LinuxPerCPUHashMap, MapSpec, MapSpecToLinuxMap, MapType, MimicError, NewLinuxEmulator, NewVM, OptMaxTailCalls, Process,
                 ProgramSpec, UnmarshalContextJSON, VM, VMOptDevice, VMOptEmulator, VMOptExecMode, VMOptSetvCPUs, VMOptShard, VMOptSpread,
                 XDPBatch, XDPResults)
from ._lib import STATUS, STATUS_NAMES, SCHED_CHUNKED, SCHED_EXPLICIT, SCHED_INTERLEAVED

__all__ = [n for n in dir() if not n.startswith("_")]
