"""One Xception entry block as ONE persistent HIP launch (entry_block.hip).

    block input x -> SepConv1 (+BN, ReLU) -> SepConv2 (+BN) -> 3x3/2 'same' max-pool
                  + BN(1x1/2 residual conv of x)  -> block output

Keras graph: ``/root/reference/guide.md:222-229`` (the served Xception); the unfused lowering is
four launches (two fused separable convs, the residual conv, pool_add). The kernel keeps both
separable-conv outputs in LDS rolling windows, so they never reach HBM.

Host side: the packed weights come from the block's three ``ConvGemmLayer`` objects (the same
BN-folded fragments the unfused kernels use); ``plan`` deals the (image, strip, pooled row)
work items out to one workgroup per CU as contiguous runs and writes the per-workgroup step
table the kernel walks (each run starts with two warm-up steps that fill the windows).
"""
from __future__ import annotations

import torch

from . import _lib
from .conv import MODE_DW, MODE_PW, ConvGemmLayer

# mode of a step (EntryBlockArgs.steps[i].w)
WARM_Y1, WARM_Y2, OUT = 0, 1, 2
MAX_STEPS = 128          # entry_block.hip EB_MAX_STEPS: a workgroup's step table lives in LDS


def entry_block_config(cfg: int) -> tuple[int, int, int, int, int]:
    """(C0, C1, PC, LDS bytes, workgroups per CU) of a kernel config (mirror of KDL_EB_CONFIGS)."""
    return tuple(_lib.lib().entry_block_config(cfg))


# kernel config per (block input channels, block output channels): entry_block.hip KDL_EB_CONFIGS
CONFIGS = {(64, 128): 0, (128, 256): 1}


def supported(cin: int, cout: int) -> bool:
    return (cin, cout) in CONFIGS


def plan_steps(B: int, OH: int, OW: int, pc: int, grid: int) -> tuple[list[tuple[int, int, int, int]], list[int]]:
    """Step table + per-workgroup offsets. Work items (image, strip, pooled row) in row-major
    order are split into ``grid`` near-equal contiguous ranges; each maximal same-(image, strip)
    run of a range is preceded by its two warm-up steps."""
    ns = (OW + pc - 1) // pc
    n = B * ns * OH
    grid = max(1, min(grid, n))
    steps: list[tuple[int, int, int, int]] = []
    off = [0]
    for g in range(grid):
        t0, t1 = g * n // grid, (g + 1) * n // grid
        t = t0
        while t < t1:
            bs, p0 = divmod(t, OH)
            p1 = min(OH, p0 + (t1 - t))
            b, s = divmod(bs, ns)
            steps.append((b, s, p0 - 2, WARM_Y1))
            steps.append((b, s, p0 - 1, WARM_Y2))
            steps.extend((b, s, p, OUT) for p in range(p0, p1))
            t += p1 - p0
        off.append(len(steps))
    return steps, off


def fit_plan(B: int, OH: int, OW: int, pc: int, wave: int) -> tuple[list[tuple[int, int, int, int]], list[int]]:
    """plan_steps on ``wave`` workgroups (one resident wave), or on as many whole waves as it
    takes for every workgroup's step table to fit EB_MAX_STEPS (large buckets: batch 128 needs
    two waves for block2). Workgroups of later waves start as earlier ones retire: the kernel
    has no inter-workgroup synchronisation, so any grid is correct."""
    grid = wave
    while True:
        steps, off = plan_steps(B, OH, OW, pc, grid)
        if max(b - a for a, b in zip(off, off[1:])) <= MAX_STEPS or grid >= B * OH * ((OW + pc - 1) // pc):
            return steps, off
        grid += wave


class EntryBlock:
    """An entry block lowered to one entry_block launch (kernel config ``cfg``)."""

    def __init__(self, name: str, sep1: ConvGemmLayer, sep2: ConvGemmLayer, res: ConvGemmLayer, cfg: int | None = None,
                 device="cuda", grid: int | None = None):
        """``grid``: workgroups (default: one per CU); ``cfg``: kernel config (default: by channels)."""
        cfg = CONFIGS[(sep1.cin_pad, sep1.n)] if cfg is None else cfg
        c0, c1, pc, lds, occ = entry_block_config(cfg)
        assert sep1.mode == MODE_DW and sep2.mode == MODE_DW and res.mode == MODE_PW and res.stride == 2, name
        assert sep1.cin_pad == c0 and sep1.n == c1 and sep2.cin_pad == c1 and sep2.n == c1, (name, c0, c1)
        assert res.cin_pad == c0 and res.n == c1 and not sep2.relu_in and sep1.relu_out == 1 and sep2.relu_out == 0
        self.name, self.cfg, self.c0, self.c1, self.pc, self.lds, self.occ = name, cfg, c0, c1, pc, lds, occ
        self.relu_in = bool(sep1.relu_in)
        assert self.relu_in == (c0 == 128), "block2 (64 -> 128): no pre-activation; block3 (128 -> 256): ReLU first"
        self.sep1, self.sep2, self.res = sep1, sep2, res
        self.device = torch.device(device)
        self.grid = grid
        self._plans: dict[tuple, tuple[torch.Tensor, torch.Tensor, int]] = {}

    def plan(self, B: int, OH: int, OW: int) -> tuple[torch.Tensor, torch.Tensor, int]:
        key = (B, OH, OW)
        if key not in self._plans:
            if self.grid:                    # an explicit grid must fit as given
                steps, off = plan_steps(B, OH, OW, self.pc, self.grid)
            else:                            # default: resident waves of workgroups, as many as fit
                steps, off = fit_plan(B, OH, OW, self.pc, self.occ * _lib.num_cus(self.device))
            assert max(b - a for a, b in zip(off, off[1:])) <= MAX_STEPS, "workgroup step table > EB_MAX_STEPS"
            st = torch.tensor(steps, dtype=torch.int32).reshape(-1, 4).to(self.device)
            of = torch.tensor(off, dtype=torch.int32).to(self.device)
            self._plans[key] = (st, of, len(off) - 1)
        return self._plans[key]

    def args(self, x: int, y: int, B: int, H: int, W: int) -> dict:
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        st, of, grid = self.plan(B, OH, OW)
        return dict(x=x, y=y, w1=_lib.ptr(self.sep1.wp), b1=_lib.ptr(self.sep1.bias), dw1=_lib.ptr(self.sep1.dww),
                    w2=_lib.ptr(self.sep2.wp), b2=_lib.ptr(self.sep2.bias), dw2=_lib.ptr(self.sep2.dww),
                    dwk1=_lib.ptr(self.sep1.dwk), dwk2=_lib.ptr(self.sep2.dwk),
                    wr=_lib.ptr(self.res.wp), br=_lib.ptr(self.res.bias), B=B, H=H, W=W, OH=OH, OW=OW,
                    ldx=self.c0, ldy=self.c1, grid=grid, steps=_lib.ptr(st), step_off=_lib.ptr(of))

    def emit(self, prog, x: int, y: int, B: int, H: int, W: int) -> None:
        a = self.args(x, y, B, H, W)
        if prog is None:
            _lib.lib().entry_block(self.cfg, a, _lib.stream_ptr())
        else:
            prog.add_entry_block(self.name, self.cfg, a)
