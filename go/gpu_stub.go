//go:build !mimic_gpu
// +build !mimic_gpu

// gpu_stub.go -- mimic built without the MI355X engine (no `-tags mimic_gpu`): the hooks the
// patches add to vm.go / emulator_linux_.go are no-ops, VMOptGPU refuses at NewVM, and RunBatch is
// the reference's own per-process loop.  See gpu.go.
package mimic

import (
	"context"

	"github.com/cilium/ebpf"
)

// GPUSettings selects the device a VM runs on.
type GPUSettings struct {
	Device int
}

// VMOptGPU runs the VM's processes on an MI355X; this build has no engine, so NewVM panics with it
// (as the reference's NewVM panics without an emulator, vm.go:73).
func VMOptGPU(device int) VMOpt {
	return func(v *VMSettings) {
		v.GPU = &GPUSettings{Device: device}
	}
}

type gpuVM struct{}

type gpuProcess struct{}

type gpuProgram struct{}

func newGPUVM(vm *VM) *gpuVM {
	if vm.settings.GPU != nil {
		panic("mimic: VMOptGPU needs a build with -tags mimic_gpu")
	}
	return nil
}

func (g *gpuVM) addMap(vm *VM, name string, m LinuxMap) (LinuxMap, error)     { return m, nil }
func (g *gpuVM) capture(prog *ebpf.ProgramSpec) *gpuProgram                     { return nil }
func (g *gpuVM) addProgram(prog *ebpf.ProgramSpec, p *gpuProgram) error        { return nil }
func (g *gpuVM) newProcess(p *Process, entrypoint int) error                  { return nil }
func (gp *gpuProcess) setCPU(id int) error                                    { return nil }
func (gp *gpuProcess) step(p *Process) (bool, error)                          { return false, nil }
func (gp *gpuProcess) run(ctx context.Context, p *Process) error              { return nil }
func (gp *gpuProcess) free()                                                  {}

// RunBatch runs one process per context: NewProcess + SetCPUID + Run + R0 + Cleanup each
// (vm.go:198-374).  With the engine (gpu.go) this is one device launch.
func (vm *VM) RunBatch(entrypoint int, ctxs []*LinuxContextXDP, cpus []int) (r0 []uint64, errs []error, err error) {
	r0 = make([]uint64, len(ctxs))
	errs = make([]error, len(ctxs))
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
