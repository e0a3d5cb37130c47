//go:build mimic_gpu
// +build mimic_gpu

// gpu.go -- the MI355X engine behind mimic's own API (package mimic, added to the reference's
// package next to vm.go).  With `-tags mimic_gpu` and VMOptGPU(device) a VM keeps its maps,
// programs and processes in libmimic_amd (include/mimic_amd.h) and every hook the patches in this
// directory add to vm.go / emulator_linux_.go forwards here; the public signatures of mimic stay
// exactly those of the reference (vm.go:54,98,198,268,291,343,363, emulator_linux_.go:97).
// Without the tag gpu_stub.go is compiled instead and mimic behaves as before.
package mimic

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#cgo LDFLAGS: -L${SRCDIR}/../mimic_amd -lmimic_amd -Wl,-rpath,${SRCDIR}/../mimic_amd
#include <stdlib.h>
#include <string.h>
#include "mimic_amd.h"
*/
import "C"

import (
	"context"
	"errors"
	"fmt"
	"syscall"
	"time"
	"unsafe"

	"github.com/cilium/ebpf"
	"github.com/cilium/ebpf/asm"
	"github.com/cilium/ebpf/btf"
)

// GPUSettings selects the device a VM runs on.
type GPUSettings struct {
	Device int
}

// VMOptGPU runs the VM's processes on an MI355X (HIP device ordinal `device`).
func VMOptGPU(device int) VMOpt {
	return func(v *VMSettings) {
		v.GPU = &GPUSettings{Device: device}
	}
}

type gpuVM struct {
	h      *C.mimic_vm
	err    error // a failed NewVM: reported by AddProgram / NewProcess (NewVM returns no error)
	mapIDs map[string]uint32
	progs  []uint32
}

type gpuProcess struct {
	vm *gpuVM
	h  *C.mimic_process
}

// gpuProgram holds a program's ELF-form slots and map relocations, captured before AddProgram
// rewrites it (the engine applies the same rewrite with the same layout, emulator_linux_.go:292-339).
type gpuProgram struct {
	raw    []byte
	relocs []C.mimic_reloc
	err    error
}

var errGPUNoLib = errors.New("libmimic_amd ABI version differs from mimic_amd.h")

func newGPUVM(vm *VM) *gpuVM {
	s := vm.settings
	if s.GPU == nil {
		return nil
	}
	g := &gpuVM{mapIDs: make(map[string]uint32)}
	if C.mimic_abi_version() != C.MIMIC_ABI_VERSION {
		g.err = errGPUNoLib
		return g
	}
	tail := 33 // emulator_linux_.go:78
	if le, ok := s.Emulator.(*LinuxEmulator); ok {
		tail = le.settings.MaxTailCalls
	}
	cs := C.mimic_vm_settings{
		vcpus:             C.int32_t(s.VirtualCPUs),
		stack_frame_size:  C.int32_t(s.StackFrameSize),
		stack_frame_count: C.int32_t(s.StackFrameCount),
		max_tail_calls:    C.int32_t(tail),
		device:            C.int32_t(s.GPU.Device),
	}
	if rc := C.mimic_vm_create(&cs, &g.h); rc != 0 {
		g.err = fmt.Errorf("mimic_vm_create: %d", int(rc))
	}
	return g
}

func (g *gpuVM) lastErr() error {
	return errors.New(C.GoString(C.mimic_last_error(g.h)))
}

// addMap: LinuxEmulator.AddMap on a GPU VM.  The map was Init'ed on the Go side (its layout entries
// match the engine's: both place entries first fit in the same order); the engine gets the same map
// with the Go map's current contents, and emu.Maps[name] becomes a LinuxMap forwarding to it.
func (g *gpuVM) addMap(vm *VM, name string, m LinuxMap) (LinuxMap, error) {
	if g.err != nil {
		return nil, g.err
	}
	spec := m.GetSpec()
	cname := C.CString(name)
	defer C.free(unsafe.Pointer(cname))
	cs := C.mimic_map_spec{name: cname, _type: C.uint32_t(spec.Type), key_size: C.uint32_t(spec.KeySize),
		value_size: C.uint32_t(spec.ValueSize), max_entries: C.uint32_t(spec.MaxEntries)}
	if _, ok := spec.Value.(*btf.Datasec); ok {
		cs.flags = C.MIMIC_MAP_F_DATASEC
	}
	var id C.uint32_t
	if C.mimic_map_create(g.h, &cs, &id) != 0 {
		return nil, g.lastErr()
	}
	g.mapIDs[name] = uint32(id)
	gm := &gpuLinuxMap{vm: g, id: uint32(id), inner: m}
	// the Go map's contents so far (datasec initial values, or Updates made before AddMap)
	for cpu := 0; cpu < m.Indices(); cpu++ {
		keys := m.Keys(cpu)
		ks := int(spec.KeySize)
		for off := 0; ks > 0 && off+ks <= len(keys); off += ks {
			key := keys[off : off+ks]
			addr, err := m.Lookup(key, cpu)
			if err != nil || addr == 0 {
				continue
			}
			entry, eoff, found := vm.MemoryController.GetEntry(addr)
			mem, isMem := entry.Object.(VMMem)
			if !found || !isMem {
				continue
			}
			val := make([]byte, spec.ValueSize)
			if mem.Read(eoff, val) != nil {
				continue
			}
			if err := gm.Update(key, val, 0, cpu); err != nil {
				return nil, err
			}
		}
	}
	return gm, nil
}

// capture: the program as the ELF has it, before AddProgram's Nop padding and rewrite.
func (g *gpuVM) capture(prog *ebpf.ProgramSpec) *gpuProgram {
	if g == nil {
		return nil
	}
	p := &gpuProgram{}
	slot := 0
	for _, ins := range prog.Instructions {
		if ins.IsLoadFromMap() {
			id, ok := g.mapIDs[ins.Reference()]
			if !ok {
				p.err = fmt.Errorf("program references a map named '%s', no map with that name exists in the emulator",
					ins.Reference())
				return p
			}
			p.relocs = append(p.relocs, C.mimic_reloc{slot: C.uint32_t(slot), map_id: C.uint32_t(id)})
		}
		var buf bytesWriter
		if _, err := ins.Marshal(&buf, asm.LittleEndian); err != nil {
			p.err = err
			return p
		}
		p.raw = append(p.raw, buf.b...)
		slot += int(ins.Size() / asm.InstructionSize)
	}
	return p
}

type bytesWriter struct{ b []byte }

func (w *bytesWriter) Write(p []byte) (int, error) {
	w.b = append(w.b, p...)
	return len(p), nil
}

// addProgram: VM.AddProgram on a GPU VM (after the Go side accepted the program).
func (g *gpuVM) addProgram(prog *ebpf.ProgramSpec, p *gpuProgram) error {
	if g.err != nil {
		return g.err
	}
	if p.err != nil {
		return p.err
	}
	if len(p.raw) == 0 {
		return errors.New("empty program")
	}
	name := C.CString(prog.Name)
	defer C.free(unsafe.Pointer(name))
	var rp *C.mimic_reloc
	if len(p.relocs) > 0 {
		rp = &p.relocs[0]
	}
	var id C.uint32_t
	if C.mimic_program_load(g.h, name, unsafe.Pointer(&p.raw[0]), C.uint32_t(len(p.raw)/8), rp,
		C.uint32_t(len(p.relocs)), &id) != 0 {
		return g.lastErr()
	}
	g.progs = append(g.progs, uint32(id))
	return nil
}

func cbytes(b []byte) unsafe.Pointer {
	if len(b) == 0 {
		return nil
	}
	return unsafe.Pointer(&b[0])
}

// newProcess: VM.NewProcess on a GPU VM -- the context's Load runs on the device
// (context_xdp_md.go:47-115, context_sk_buff.go:42-107).
func (g *gpuVM) newProcess(p *Process, entrypoint int) error {
	if g.err != nil {
		return g.err
	}
	prog := C.uint32_t(g.progs[entrypoint])
	gp := &gpuProcess{vm: g}
	switch c := p.Context.(type) {
	case *LinuxContextXDP:
		if C.mimic_process_new(g.h, prog, cbytes(c.Packet), C.uint32_t(len(c.Packet)), C.uint32_t(c.Headroom),
			C.uint32_t(c.Tailroom), C.int32_t(c.IngessIfIndex), C.int32_t(c.RxQueueIndex), C.int32_t(c.EgressIfIndex),
			&gp.h) != 0 {
			return fmt.Errorf("context load: %w", g.lastErr())
		}
	case *LinuxContextSKBuff:
		var ifindex uint32
		if c.Dev != nil {
			ifindex = c.Dev.IFIndex
		}
		var cust C.mimic_skb_custom
		skbCustom(c, &cust)
		if C.mimic_process_new_skb_ctx(g.h, prog, cbytes(c.Packet), C.uint32_t(len(c.Packet)), C.uint32_t(ifindex),
			&cust, &gp.h) != 0 {
			return fmt.Errorf("context load: %w", g.lastErr())
		}
	default:
		return fmt.Errorf("context load: a GPU VM runs xdp_md and sk_buff contexts, not %T", p.Context)
	}
	p.gpu = gp
	return nil
}

// skbCustom: a user-given SK / FlowKeys (context_sk_buff.go:53-66) as the engine's entry
// (include/mimic_amd.h mimic_skb_custom); flags 0 when the context gives neither.
func skbCustom(c *LinuxContextSKBuff, out *C.mimic_skb_custom) {
	if sk := c.SK; sk != nil {
		out.flags |= C.MIMIC_SKB_CUSTOM_SK
		out.sk_bound_dev_if = C.uint32_t(sk.BoundDevIF)
		out.sk_family = C.uint32_t(sk.Family)
		out.sk_type = C.uint32_t(sk.SockType)
		out.sk_protocol = C.uint32_t(sk.Protocol)
		out.sk_mark = C.uint32_t(sk.Mark)
		out.sk_priority = C.uint32_t(sk.Priority)
		out.sk_src_port = C.uint32_t(sk.SrcPort)
		out.sk_dst_port = C.uint32_t(sk.DstPort)
		out.sk_state = C.uint32_t(sk.State)
		out.sk_rx_queue_mapping = C.int32_t(sk.RXQueueMapping)
		for i, ip := range [][]byte{sk.srcIP4, sk.dstIP4, sk.srcIP6, sk.dstIP6} {
			n := len(ip)
			if n > 16 {
				n = 16
			}
			out.sk_ip_len[i] = C.uint8_t(n)
			for j := 0; j < n; j++ {
				out.sk_ip[i][j] = C.uint8_t(ip[j])
			}
		}
	}
	if fk := c.FlowKeys; fk != nil {
		out.flags |= C.MIMIC_SKB_CUSTOM_FLOWKEYS
		out.fk_nhoff = C.uint16_t(fk.Nhoff)
		out.fk_thoff = C.uint16_t(fk.Thoff)
		out.fk_addr_proto = C.uint16_t(fk.AddrProto)
		out.fk_is_frag = C.uint8_t(fk.IsFrag)
		out.fk_is_first_frag = C.uint8_t(fk.IsFirstFrag)
		out.fk_is_encap = C.uint8_t(fk.IsEncap)
		out.fk_ip_proto = C.uint8_t(fk.IPProto)
		out.fk_n_proto = C.uint16_t(fk.NProto)
		out.fk_sport = C.uint16_t(fk.Sport)
		out.fk_dport = C.uint16_t(fk.Dport)
		out.fk_flags = C.uint32_t(fk.Flags)
		out.fk_flow_label = C.uint32_t(fk.FlowLabel)
	}
}

func (gp *gpuProcess) setCPU(id int) error {
	if C.mimic_process_set_cpu(gp.h, C.int32_t(id)) != 0 {
		return gp.vm.lastErr()
	}
	return nil
}

// take copies the engine's registers into p.Registers (vm.go:377-404)
func (gp *gpuProcess) take(p *Process, r *C.mimic_process_regs) {
	p.Registers = Registers{
		PC: int(r.pc), R0: uint64(r.r[0]), R1: uint64(r.r[1]), R2: uint64(r.r[2]), R3: uint64(r.r[3]),
		R4: uint64(r.r[4]), R5: uint64(r.r[5]), R6: uint64(r.r[6]), R7: uint64(r.r[7]), R8: uint64(r.r[8]),
		R9: uint64(r.r[9]), R10: uint64(r.r[10]),
	}
}

func statusErr(r *C.mimic_process_regs) error {
	return fmt.Errorf("inst at PC(%d): engine status %d", int(r.pc), int(r.status))
}

// step: Process.Step (vm.go:291-340) -- one instruction on the device.
func (gp *gpuProcess) step(p *Process) (bool, error) {
	var r C.mimic_process_regs
	if rc := C.mimic_process_step(gp.h, 1, &r); rc != 0 {
		gp.take(p, &r)
		return true, gp.vm.lastErr() // "process has been terminated"
	}
	gp.take(p, &r)
	if r.status != 0 { // MIMIC_OK
		return true, statusErr(&r)
	}
	return r.exited != 0, nil
}

// run: Process.Run(ctx) (vm.go:343-360) -- one launch per slice, ctx checked between slices and
// by the kernel every 4096 steps; p.Registers hold R0-R10 and PC afterwards.
func (gp *gpuProcess) run(ctx context.Context, p *Process) error {
	var r C.mimic_process_regs
	var rc C.int
	if ctx.Done() == nil { // context.Background() / TODO(): never done
		rc = C.mimic_process_run(gp.h, 0, &r)
	} else {
		c, done := gpuCtx(ctx)
		rc = C.mimic_process_run_ctx(gp.h, 0, c, &r)
		done()
	}
	gp.take(p, &r)
	switch {
	case rc == C.MIMIC_ECANCELED || rc == C.MIMIC_EDEADLINE:
		return ctx.Err()
	case rc != 0:
		return fmt.Errorf("process encountered a fatal error: %w", gp.vm.lastErr())
	case r.status != 0: // MIMIC_OK
		return fmt.Errorf("process encountered a fatal error: %w", statusErr(&r))
	}
	return nil
}

func (gp *gpuProcess) free() {
	C.mimic_process_free(gp.h)
	gp.h = nil
}

// gpuCtx turns a context.Context into the engine's context word (pinned host memory the kernels
// read); the returned func frees it once the runs that use it returned.
func gpuCtx(ctx context.Context) (*C.mimic_ctx, func()) {
	var c *C.mimic_ctx
	var ns C.uint64_t
	if d, ok := ctx.Deadline(); ok {
		left := time.Until(d).Nanoseconds()
		if left < 1 {
			left = 1
		}
		ns = C.uint64_t(left)
	}
	C.mimic_ctx_new(ns, &c)
	stop := make(chan struct{})
	go func() {
		select {
		case <-ctx.Done():
			if ctx.Err() == context.Canceled {
				C.mimic_ctx_cancel(c)
			} // DeadlineExceeded: the engine's own timer marks it
		case <-stop:
		}
	}()
	return c, func() { close(stop); C.mimic_ctx_free(c) }
}

// RunBatch runs one process per context as ONE device launch: for each i, NewProcess(entrypoint,
// ctxs[i]) + SetCPUID(cpus[i]) + Run + R0 + Cleanup (vm.go:198-374), a vCPU's processes in slice
// order (processPool's per-worker order, vm.go:548-573).  The contexts share Headroom, Tailroom
// and the interface indexes (the engine's host batch takes them once); packet bytes the program
// wrote are copied back into ctxs[i].Packet.  errs[i] is what Run returned for process i.  Not in
// the reference API; on a VM without VMOptGPU it runs the processes one by one.
func (vm *VM) RunBatch(entrypoint int, ctxs []*LinuxContextXDP, cpus []int) (r0 []uint64, errs []error, err error) {
	if len(ctxs) != len(cpus) {
		return nil, nil, errors.New("one cpu per context")
	}
	g := vm.gpu
	if g == nil {
		return vm.runBatchHost(entrypoint, ctxs, cpus)
	}
	if g.err != nil {
		return nil, nil, g.err
	}
	if entrypoint < 0 || entrypoint >= len(g.progs) {
		return nil, nil, fmt.Errorf("no program with id '%d' is loaded", entrypoint)
	}
	n := len(ctxs)
	if n == 0 {
		return nil, nil, nil
	}
	c0 := ctxs[0]
	off := make([]uint64, n)
	lens := make([]uint32, n)
	cpu := make([]int32, n)
	var total uint64
	for i, c := range ctxs {
		if c.Headroom != c0.Headroom || c.Tailroom != c0.Tailroom || c.IngessIfIndex != c0.IngessIfIndex ||
			c.RxQueueIndex != c0.RxQueueIndex || c.EgressIfIndex != c0.EgressIfIndex {
			return nil, nil, fmt.Errorf("context %d: RunBatch contexts share headroom, tailroom and interfaces", i)
		}
		off[i] = total
		lens[i] = uint32(len(c.Packet))
		cpu[i] = int32(cpus[i])
		total += (uint64(c.Headroom+len(c.Packet)+c.Tailroom) + 63) &^ 63
	}
	buf := make([]byte, total)
	for i, c := range ctxs {
		copy(buf[off[i]+uint64(c.Headroom):], c.Packet)
	}
	r0 = make([]uint64, n)
	status := make([]uint8, n)
	hb := C.mimic_xdp_host_batch{
		n: C.uint32_t(n), schedule: C.MIMIC_SCHED_EXPLICIT, pkt_data: (*C.uint8_t)(cbytes(buf)),
		pkt_off: (*C.uint64_t)(unsafe.Pointer(&off[0])), pkt_len: (*C.uint32_t)(unsafe.Pointer(&lens[0])),
		headroom_all: C.uint32_t(c0.Headroom), tailroom_all: C.uint32_t(c0.Tailroom),
		ingress_all: C.int32_t(c0.IngessIfIndex), rxq_all: C.int32_t(c0.RxQueueIndex), egress_all: C.int32_t(c0.EgressIfIndex),
		cpu: (*C.int32_t)(unsafe.Pointer(&cpu[0])), pkt_out: (*C.uint8_t)(cbytes(buf)),
		r0: (*C.uint64_t)(unsafe.Pointer(&r0[0])), status: (*C.uint8_t)(unsafe.Pointer(&status[0])),
	}
	if C.mimic_run_xdp_host(g.h, C.uint32_t(g.progs[entrypoint]), &hb, 0) != 0 {
		return nil, nil, g.lastErr()
	}
	errs = make([]error, n)
	for i, c := range ctxs {
		copy(c.Packet, buf[off[i]+uint64(c.Headroom):])
		if status[i] != 0 { // MIMIC_OK
			errs[i] = fmt.Errorf("process encountered a fatal error: engine status %d", int(status[i]))
		}
	}
	return r0, errs, nil
}

// runBatchHost: RunBatch's meaning on a Go-only VM (the reference's own loop).
func (vm *VM) runBatchHost(entrypoint int, ctxs []*LinuxContextXDP, cpus []int) ([]uint64, []error, error) {
	r0 := make([]uint64, len(ctxs))
	errs := make([]error, len(ctxs))
	for i, c := range ctxs {
		p, err := vm.NewProcess(entrypoint, c)
		if err != nil {
			return nil, nil, err
		}
		if err = p.SetCPUID(cpus[i]); err == nil {
			err = p.Run(context.Background())
		}
		r0[i], errs[i] = p.Registers.R0, err
		_ = p.Cleanup()
	}
	return r0, errs, nil
}

// gpuLinuxMap is emu.Maps[name] on a GPU VM: host map operations on the engine's copy
// (emulator_linux_map.go:14-42; hash maps run on a host image of the device index, no device round
// trip per call).
type gpuLinuxMap struct {
	vm    *gpuVM
	id    uint32
	inner LinuxMap
}

var (
	_ LinuxMap        = (*gpuLinuxMap)(nil)
	_ LinuxMapUpdater = (*gpuLinuxMap)(nil)
	_ LinuxMapDeleter = (*gpuLinuxMap)(nil)
)

func (m *gpuLinuxMap) Init(emulator *LinuxEmulator) error { return nil }

func (m *gpuLinuxMap) GetSpec() ebpf.MapSpec { return m.inner.GetSpec() }

func (m *gpuLinuxMap) Indices() int { return m.inner.Indices() }

func (m *gpuLinuxMap) Keys(cpuid int) []byte {
	spec := m.inner.GetSpec()
	out := make([]byte, int(spec.MaxEntries)*int(spec.KeySize))
	var n C.uint32_t
	if C.mimic_map_keys(m.vm.h, C.uint32_t(m.id), cbytes(out), C.size_t(len(out)), &n) != 0 {
		return nil
	}
	return out[:int(n)*int(spec.KeySize)]
}

func (m *gpuLinuxMap) Lookup(key []byte, cpuid int) (uint32, error) {
	var addr C.uint32_t
	if rc := C.mimic_map_lookup(m.vm.h, C.uint32_t(m.id), cbytes(key), C.int32_t(cpuid), &addr); rc < 0 {
		return 0, m.vm.lastErr()
	} else if rc > 0 {
		return 0, syscall.Errno(rc)
	}
	return uint32(addr), nil
}

func (m *gpuLinuxMap) Update(key []byte, value []byte, flags uint32, cpuid int) error {
	rc := C.mimic_map_update(m.vm.h, C.uint32_t(m.id), cbytes(key), cbytes(value), C.uint32_t(flags), C.int32_t(cpuid))
	switch {
	case rc < 0:
		return m.vm.lastErr()
	case rc > 0:
		return syscall.Errno(rc) // graceful: forwarded to the program as the reference does
	}
	return nil
}

func (m *gpuLinuxMap) Delete(key []byte) error {
	rc := C.mimic_map_delete(m.vm.h, C.uint32_t(m.id), cbytes(key))
	switch {
	case rc < 0:
		return m.vm.lastErr()
	case rc > 0:
		return syscall.Errno(rc)
	}
	return nil
}

// Values returns the value backing of (map, cpuid) as the device has it: E*S bytes in slot order.
func (m *gpuLinuxMap) Values(cpuid int) ([]byte, error) {
	spec := m.inner.GetSpec()
	out := make([]byte, int(spec.MaxEntries)*int(spec.ValueSize))
	if C.mimic_map_read_values(m.vm.h, C.uint32_t(m.id), C.int32_t(cpuid), cbytes(out), C.size_t(len(out))) != 0 {
		return nil, m.vm.lastErr()
	}
	return out, nil
}
