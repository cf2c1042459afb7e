#!/usr/bin/env python
"""Dump the gfx950 disassembly of the kernels of a built library whose demangled name matches
a regex (the ISA audits behind profiles/*: waitcnt placement, register counts).
  python tools/kasm.py kdl/_C.cpython-310-x86_64-linux-gnu.so 'sepconv_ws_kernel<6, 6, 5, 9, false, true, false, 0, false>'
"""
from __future__ import annotations

import re
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from vmcnt_check import LLVM, disassemble  # noqa: E402


def main() -> int:
    lib, pat = Path(sys.argv[1]), re.compile(sys.argv[2])
    for k in disassemble(lib):
        name = subprocess.run(["c++filt"], input=k.name, capture_output=True, text=True).stdout.strip()
        if pat.search(name):
            print(f"== {name} ({len(k.insns)} instructions)")
            for i in k.insns:
                print(f"{i.addr:6x}  {i.text}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
