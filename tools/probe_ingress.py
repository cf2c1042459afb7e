"""Ingress-overlap probe: graph only / serial H2D / overlapped H2D (copy stream)."""
import sys, time, torch, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from kdl.engine import registry
from kdl.engine.tuning import tuning_path
model = sys.argv[1] if len(sys.argv) > 1 else "xception"
info = registry.get(model)
eng = info.engine(info.init_params(0), 32, torch.device('cuda', 0))
eng.load_tuning(tuning_path(model, 32))
S = info.input_size
slots = eng.add_input_slots(2)
host = torch.randint(0, 256, (32, S, S, 3), dtype=torch.uint8).pin_memory()
s, cs = eng.stream, torch.cuda.Stream()
ev = [torch.cuda.Event() for _ in range(4)]
def run(mode, n=60):
    for i in range(n + 5):
        if i == 5:
            torch.cuda.synchronize(); t0 = time.perf_counter()
        j = i % 2
        if mode == "graph":
            eng.launch(32, s, slot=j)
        elif mode == "serial":
            with torch.cuda.stream(s):
                slots[j].copy_(host, non_blocking=True)
            eng.launch(32, s, slot=j)
        elif mode in ("overlap", "overlap_sdma_off"):
            with torch.cuda.stream(cs):
                cs.wait_event(ev[2 + j])
                slots[j].copy_(host, non_blocking=True)
                ev[j].record(cs)
            s.wait_event(ev[j])
            eng.launch(32, s, slot=j)
            ev[2 + j].record(s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3
for _ in range(2):
    for m in ("graph", "serial", "overlap"):
        print(f"{model} {m:8s} {run(m):.3f} ms/step", flush=True)
