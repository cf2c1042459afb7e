import sys, time, torch
sys.path.insert(0, '.')
from kdl.engine import registry
info = registry.get('resnet50')
p = info.init_params(0)
eng = info.engine(p, 32, torch.device('cuda', 0))
from kdl.engine.tuning import tuning_path
import os
eng.load_tuning('gpurun_out/resnet50_b32.json') if os.path.exists('gpurun_out/resnet50_b32.json') else None
for _ in range(5): eng.launch(32)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100): eng.launch(32)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"graph-only: cpu submit {(t1-t0)*10:.3f} ms/launch, wall {(t2-t0)*10:.3f} ms/step")
s = eng.stream
x = torch.randint(0, 256, (32, 224, 224, 3), dtype=torch.uint8).pin_memory()
st = torch.empty_like(x, device='cuda')
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100):
    with torch.cuda.stream(s):
        st.copy_(x, non_blocking=True)
torch.cuda.synchronize()
print(f"H2D 4.8MB: {(time.perf_counter()-t0)*10:.3f} ms")
