"""The Go binding keeps mimic's own surface (go/: gpu.go, gpu_stub.go, mimic_gpu.patch).  No Go
toolchain exists in this image, so the binding is checked structurally:

* the patch applies to the reference's vm.go / emulator_linux_.go and only ADDS lines;
* every exported func of the patched vm.go has exactly the reference's signature
  (NewVM vm.go:54, AddProgram :98, NewProcess :198, SetCPUID :268, Step :291, Run :343, Cleanup :363)
  and every reference struct field is still there;
* the hooks the patch adds call methods that gpu.go (engine build) and gpu_stub.go (default build)
  both define with the same parameters;
* every C function gpu.go calls is declared in include/mimic_amd.h with that many parameters, and
  every C struct field it sets exists there; the context fields it reads exist in the reference's
  LinuxContextXDP / LinuxContextSKBuff / SK / FlowKeys / NetDev.
The reference is read only where it is present (this container), never on the GPU box."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go")
REF = "/root/reference"
HDR = os.path.join(ROOT, "include", "mimic_amd.h")
have_ref = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "vm.go")), reason="reference not present")


def _read(p):
    with open(p) as f:
        return f.read()


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _funcs(src):
    """name -> signature line (receiver, params, results) of every top-level func."""
    out = {}
    for m in re.finditer(r"^func (\([^)]*\) )?(\w+)\((.*)\s*\{\s*$", src, flags=re.M):
        recv = (m.group(1) or "").strip()
        key = (re.sub(r"\(\w+ \*?", "(", recv).strip("()") if recv else "", m.group(2))
        out[key] = m.group(0).rstrip(" {\n")
    return out


def _patched(tmp_path):
    for f in ("vm.go", "emulator_linux_.go"):
        shutil.copy(os.path.join(REF, f), tmp_path / f)
    r = subprocess.run(["patch", "-p1", "--no-backup-if-mismatch", "-i", os.path.join(GO, "mimic_gpu.patch")],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return _read(tmp_path / "vm.go"), _read(tmp_path / "emulator_linux_.go")


def test_patch_only_adds_lines():
    patch = _read(os.path.join(GO, "mimic_gpu.patch"))
    files = re.findall(r"^\+\+\+ b/(\S+)", patch, flags=re.M)
    assert files == ["vm.go", "emulator_linux_.go"]
    removed = [l for l in patch.splitlines() if l.startswith("-") and not l.startswith("---")]
    assert removed == [], removed


@have_ref
def test_patched_vm_keeps_the_reference_signatures(tmp_path):
    vm_new, emu_new = _patched(tmp_path)
    ref = _funcs(_read(os.path.join(REF, "vm.go")))
    new = _funcs(vm_new)
    exported = {k: v for k, v in ref.items() if k[1][0].isupper()}
    for k, sig in exported.items():
        assert new.get(k) == sig, (k, sig, new.get(k))
    assert set(k for k in new if k[1][0].isupper()) == set(exported)
    # the signatures the drop-in names, as the reference declares them (vm.go:54,98,198,268,291,343,363)
    want = {
        ("", "NewVM"): "func NewVM(opts ...VMOpt) *VM",
        ("VM", "AddProgram"): "func (vm *VM) AddProgram(prog *ebpf.ProgramSpec) (int, error)",
        ("VM", "NewProcess"): "func (vm *VM) NewProcess(entrypoint int, ctx Context) (*Process, error)",
        ("Process", "SetCPUID"): "func (p *Process) SetCPUID(id int) error",
        ("Process", "Step"): "func (p *Process) Step() (exited bool, err error)",
        ("Process", "Run"): "func (p *Process) Run(ctx context.Context) error",
        ("Process", "Cleanup"): "func (p *Process) Cleanup() error",
    }
    for k, sig in want.items():
        assert new[k] == sig
    ref_lines = _read(os.path.join(REF, "vm.go")).splitlines()
    for k, line in zip(want, (54, 98, 198, 268, 291, 343, 363)):
        assert ref_lines[line - 1].rstrip(" {") == want[k]
    assert _funcs(emu_new)[("LinuxEmulator", "AddMap")] == _funcs(_read(os.path.join(REF, "emulator_linux_.go")))[
        ("LinuxEmulator", "AddMap")]


def _struct_fields(src, name):
    m = re.search(r"^type " + name + r" struct \{(.*?)^\}", src, flags=re.M | re.S)
    assert m, name
    body = _strip_comments(m.group(1))
    return [l.split()[0] for l in body.splitlines() if l.strip()]


@have_ref
def test_patched_structs_keep_every_reference_field(tmp_path):
    vm_new, _ = _patched(tmp_path)
    ref = _read(os.path.join(REF, "vm.go"))
    for name in ("VMSettings", "VM", "Process"):
        old, new = _struct_fields(ref, name), _struct_fields(vm_new, name)
        assert new[:len(old)] == old, name
    assert _struct_fields(vm_new, "VMSettings")[-1] == "GPU"


def _methods(src):
    """(receiver type, name) -> normalised parameter list of the gpu* helpers."""
    out = {}
    for m in re.finditer(r"^func (?:\(\w+ \*?(\w+)\) )?(\w+)\(([^)]*)\)", _strip_comments(src), flags=re.M):
        params = re.sub(r"\s+", " ", m.group(3)).strip()
        out[(m.group(1) or "", m.group(2))] = params
    return out


def test_engine_and_stub_builds_define_the_same_hooks():
    eng = _methods(_read(os.path.join(GO, "gpu.go")))
    stub = _methods(_read(os.path.join(GO, "gpu_stub.go")))
    patch = _read(os.path.join(GO, "mimic_gpu.patch"))
    called = set(re.findall(r"\.gpu\.(\w+)\(", patch)) | set(re.findall(r"\b(newGPUVM)\(", patch))
    assert called == {"newGPUVM", "capture", "addProgram", "newProcess", "setCPU", "step", "run", "free", "addMap"}
    for name in called:
        ek = [k for k in eng if k[1] == name]
        sk = [k for k in stub if k[1] == name]
        assert len(ek) == 1 and len(sk) == 1, name
        assert ek[0] == sk[0] and eng[ek[0]] == stub[sk[0]], (name, eng[ek[0]], stub[sk[0]])
    for k in (("", "VMOptGPU"), ("VM", "RunBatch")):
        assert eng[k] == stub[k], k
    for f in ("gpu.go", "gpu_stub.go"):
        s = _strip_comments(_read(os.path.join(GO, f)))
        s = re.sub(r'"(?:\\.|[^"\\])*"', '""', s)
        assert s.count("{") == s.count("}") and s.count("(") == s.count(")"), f


def _c_protos():
    hdr = _strip_comments(_read(HDR))
    protos = {}
    for m in re.finditer(r"\b(?:int|void|long|const char \*)\s*(mimic_\w+)\(([^;]*?)\);", hdr, flags=re.S):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return protos


def _call_args(src, start):
    depth, i, n, seen = 0, start, 0, False
    while True:
        c = src[i]
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
            if depth == 0:
                return n + (1 if seen else 0)
        elif c == "," and depth == 1:
            n += 1
        elif not c.isspace() and depth >= 1:
            seen = True
        i += 1


def test_cgo_calls_match_the_header():
    src = _strip_comments(_read(os.path.join(GO, "gpu.go")))
    protos = _c_protos()
    calls = list(re.finditer(r"\bC\.(mimic_\w+)\(", src))
    assert len(calls) > 20
    for m in calls:
        name = m.group(1)
        assert name in protos, name
        assert _call_args(src, m.end() - 1) == protos[name], name
    hdr = _read(HDR)
    for m in re.finditer(r"C\.(mimic_\w+)\{(.*?)\}\s*$", src, flags=re.S | re.M):
        td = re.search(r"typedef struct \{(.*?)\}\s*" + m.group(1) + ";", hdr, flags=re.S)
        assert td, m.group(1)
        for fld in re.findall(r"(\w+):", m.group(2)):
            fld = "type" if fld == "_type" else fld
            assert re.search(r"\b" + fld + r"\b", td.group(1)), (m.group(1), fld)


@have_ref
def test_context_fields_exist_in_the_reference():
    src = _strip_comments(_read(os.path.join(GO, "gpu.go")))
    xdp = _read(os.path.join(REF, "context_xdp_md.go"))
    skb = _read(os.path.join(REF, "context_sk_buff.go")) + _read(os.path.join(REF, "emulator_linux_sk_buff.go"))
    fields = {"LinuxContextXDP": _struct_fields(xdp, "LinuxContextXDP"),
              "LinuxContextSKBuff": _struct_fields(skb, "LinuxContextSKBuff"),
              "SK": _struct_fields(skb, "SK"), "FlowKeys": _struct_fields(skb, "FlowKeys"),
              "NetDev": _struct_fields(skb, "NetDev")}
    for f in ("Headroom", "Tailroom", "Packet", "IngessIfIndex", "RxQueueIndex", "EgressIfIndex"):
        assert f in fields["LinuxContextXDP"] and f"c.{f}" in src, f
    for f in ("Packet", "SK", "Dev", "FlowKeys"):
        assert f in fields["LinuxContextSKBuff"], f
    for f in re.findall(r"\bsk\.(\w+)", src):
        assert f in fields["SK"], f
    for f in re.findall(r"\bfk\.(\w+)", src):
        assert f in fields["FlowKeys"], f
    assert "IFIndex" in fields["NetDev"]
