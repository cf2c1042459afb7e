#!/usr/bin/env python
"""Static check of in-flight vector-memory loads in gfx950 code objects.

A VMEM load (``global_load_*``, ``buffer_load_*`` without ``lds`` ...) writes its
destination VGPRs when the data RETURNS, not when it issues; the program must not
touch those registers until an ``s_waitcnt vmcnt(N)`` has retired the load. The
compiler guarantees this for loads it generates, but NOT for loads issued from
inline asm (``sepconv_ws.hip`` issues its register-resident pointwise-weight loads
that way, covered by hand-counted waits): the compiler believes the asm wrote its
output at issue, so where it regards part of that output as dead it may re-allocate
those registers -- e.g. as the ADDRESS of the next load, which the returning data
then overwrites (a wild address: GPU memory fault).

This tool disassembles every kernel of an object / shared library (its
``.hip_fatbin`` gfx950 bundle), walks each kernel's control-flow graph with a
conservative model of the in-order vmcnt queue (per path: which VGPRs each
outstanding load will still write), and reports every instruction that reads or
writes a VGPR/AGPR a load may still be writing.

    python tools/vmcnt_check.py kdl/_C.cpython-310-x86_64-linux-gnu.so [--kernel REGEX]

Exit status 1 if any hazard is found. ``tests/test_vmcnt_hazards.py`` runs it over
the built extension.
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
_INSN = re.compile(r"^\s+([a-z_0-9]+)(.*?)\s*//\s*([0-9A-F]+):")
_BR_TARGET = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
_REG = re.compile(r"\b([va])(?:(\d+)|\[(\d+):(\d+)\])")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")
VMCNT_MAX = 63


def _regs(text: str) -> int:
    """Bit mask of the VGPRs (bits 0..511) and AGPRs (bits 512..) an operand string names."""
    out = 0
    for m in _REG.finditer(text):
        off = 0 if m.group(1) == "v" else 512
        if m.group(2) is not None:
            out |= 1 << (off + int(m.group(2)))
        else:
            lo, hi = int(m.group(3)), int(m.group(4))
            out |= ((1 << (hi - lo + 1)) - 1) << (off + lo)
    return out


def _names(mask: int) -> str:
    return ",".join(("v%d" % b) if b < 512 else ("a%d" % (b - 512)) for b in range(mask.bit_length())
                    if mask >> b & 1)


@dataclass
class Insn:
    addr: int
    op: str
    args: str
    text: str

    @property
    def is_vmem(self) -> bool:
        return self.op.startswith(("global_", "buffer_", "flat_", "scratch_", "tbuffer_"))

    def load_dst(self) -> int:
        """VGPRs/AGPRs the instruction writes asynchronously (returning loads/atomics)."""
        if not self.is_vmem:
            return 0
        a = self.args.strip()
        if " lds" in f" {a} " or "_lds_" in self.op or self.op.endswith("_lds"):
            return 0
        is_load = "_load_" in self.op or self.op.endswith("_load")
        is_ret_atomic = "_atomic_" in self.op and " glc" in f" {a}"   # returning atomic
        if not (is_load or is_ret_atomic):
            return 0
        first = a.split(",")[0]
        return _regs(first)

    def touched(self) -> int:
        """Registers the instruction reads or writes synchronously. A returning load's own
        destination is excluded: VMEM loads return in issue order, so a load that
        re-targets a pending load's registers (WAW) is safe; its address operands are not."""
        if self.load_dst():
            return _regs(",".join(self.args.split(",")[1:]))
        return _regs(self.args)


@dataclass
class Kernel:
    name: str
    insns: list[Insn] = field(default_factory=list)


def disassemble(path: Path) -> list[Kernel]:
    """Kernels of a host object / .so with a HIP fat binary, or of a bare code object."""
    with tempfile.TemporaryDirectory() as td:
        fat = Path(td) / "k.fatbin"
        r = subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(path),
                            str(Path(td) / "junk")], capture_output=True, text=True)
        cos = []
        if r.returncode == 0 and fat.exists():
            # a linked .so concatenates one offload bundle per object file
            blob = fat.read_bytes()
            magic = b"__CLANG_OFFLOAD_BUNDLE__"
            starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
            for j, s in enumerate(starts):
                part = Path(td) / f"b{j}.fatbin"
                part.write_bytes(blob[s:starts[j + 1] if j + 1 < len(starts) else len(blob)])
                co = Path(td) / f"b{j}.co"
                rr = subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                                     f"--input={part}", f"--targets={TARGET}", f"--output={co}"],
                                    capture_output=True)
                if rr.returncode == 0 and co.exists() and co.stat().st_size:
                    cos.append(co)
        else:
            cos = [path]
        txt = "\n".join(subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                                       check=True, capture_output=True, text=True).stdout for co in cos)
    kernels: list[Kernel] = []
    cur = None
    for line in txt.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = Kernel(m.group(2))
            kernels.append(cur)
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if m:
            cur.insns.append(Insn(int(m.group(3), 16), m.group(1), m.group(2), line.strip()))
    return kernels


def _successors(k: Kernel, i: int, index: dict[int, int], base: dict[str, int]) -> list[int]:
    ins = k.insns[i]
    if ins.op in ("s_endpgm", "s_setpc_b64", "s_trap"):
        return []
    tgt = None
    if ins.op.startswith(("s_branch", "s_cbranch")):
        m = _BR_TARGET.search(ins.text)
        if m and m.group(1) in base:
            tgt = index.get(base[m.group(1)] + int(m.group(2), 16))
    if ins.op == "s_branch":
        return [tgt] if tgt is not None else []
    nxt = [i + 1] if i + 1 < len(k.insns) else []
    return nxt + ([tgt] if tgt is not None else [])


# queue state: tuple (oldest .. youngest) of int masks of pending destination registers
def _join(a: tuple, b: tuple) -> tuple:
    """Conservative merge of two vmcnt queues aligned at the youngest end."""
    n = max(len(a), len(b))
    a = (0,) * (n - len(a)) + a
    b = (0,) * (n - len(b)) + b
    return tuple(x | y for x, y in zip(a, b))


def _strip(q: tuple) -> tuple:
    """Drop leading (oldest) entries that write no register: they cannot cause a hazard,
    and keeping them would only make otherwise-equal states differ."""
    i = 0
    while i < len(q) and q[i] == 0:
        i += 1
    return q[i:]


def check_kernel(k: Kernel, base: dict[str, int]) -> list[str]:
    if not k.insns:
        return []
    index = {ins.addr: i for i, ins in enumerate(k.insns)}
    n = len(k.insns)
    # per instruction: (kind, arg) with kind 0 plain, 1 waitcnt (arg = N), 2 vmem (arg = dst mask)
    touch = [ins.touched() for ins in k.insns]
    kind, arg = [0] * n, [0] * n
    for i, ins in enumerate(k.insns):
        if ins.op == "s_waitcnt":
            m = _VMCNT.search(ins.args)
            kind[i], arg[i] = 1, (int(m.group(1)) if m else VMCNT_MAX)
        elif ins.is_vmem:
            kind[i], arg[i] = 2, ins.load_dst()
    succ = [_successors(k, i, index, base) for i in range(n)]
    # basic-block leaders: entry, branch targets, fall-throughs after branches
    leaders = {0}
    for i in range(n):
        if len(succ[i]) != 1 or succ[i][0] != i + 1:
            leaders.update(succ[i])
            if i + 1 < n:
                leaders.add(i + 1)
    state: dict[int, tuple] = {0: ()}
    work = {0}
    hazards: dict[int, str] = {}
    while work:
        b = min(work)             # address order: loop bodies converge in few passes
        work.discard(b)
        q = state[b]
        i = b
        while True:
            pending = 0
            for x in q:
                pending |= x
            if kind[i] == 1:
                c = arg[i]
                q = () if c == 0 else (q[len(q) - c:] if c < len(q) else q)
            else:
                hit = touch[i] & pending
                if hit and i not in hazards:
                    hazards[i] = (f"{k.name}: {k.insns[i].text.split('//')[0].strip()}  @0x{k.insns[i].addr:x} "
                                  f"touches {_names(hit)} of an in-flight load")
                if kind[i] == 2:
                    q = q + (arg[i],)
                    if len(q) > VMCNT_MAX + 1:
                        q = q[-(VMCNT_MAX + 1):]
            q = _strip(q)
            ss = succ[i]
            if len(ss) == 1 and ss[0] == i + 1 and (i + 1) not in leaders:
                i += 1
                continue
            for s in ss:
                old = state.get(s)
                new = q if old is None else _strip(_join(old, q))
                if new != old:
                    state[s] = new
                    work.add(s)
            break
    return [hazards[i] for i in sorted(hazards)]


def check(path: Path, kernel_re: str | None = None) -> tuple[int, list[str]]:
    kernels = disassemble(path)
    base = {k.name: k.insns[0].addr for k in kernels if k.insns}
    rx = re.compile(kernel_re) if kernel_re else None
    out, n = [], 0
    for k in kernels:
        if rx and not rx.search(k.name):
            continue
        n += 1
        out += check_kernel(k, base)
    return n, out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("path", type=Path)
    ap.add_argument("--kernel", default=None, help="only kernels whose (mangled) name matches this regex")
    ap.add_argument("--max", type=int, default=40, help="hazard lines to print")
    a = ap.parse_args(argv)
    n, hz = check(a.path, a.kernel)
    for h in hz[:a.max]:
        print(h)
    kn = sorted({h.split(":")[0] for h in hz})
    print(f"{n} kernels checked, {len(hz)} hazard(s) in {len(kn)} kernel(s)")
    for name in kn:
        print("  ", name)
    return 1 if hz else 0


if __name__ == "__main__":
    sys.exit(main())
