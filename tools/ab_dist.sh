# interleaved A/B of the multi-rank bench path on one GPU, one rank under torchrun:
# p = plain bench.py (no process group); g = --force-dist, native RCCL gather + gloo control group (default);
# n = native gather + an nccl control group (a second RCCL communicator); t = torch.distributed.gather (nccl)
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
bash tools/gpu_session.sh \
 p0 200 python bench.py -- \
 g0 300 $TR --master-port 29511 bench.py --gpus 1 --force-dist -- \
 n0 300 $TR --master-port 29512 bench.py --gpus 1 --force-dist --dist-backend nccl -- \
 t0 300 $TR --master-port 29513 bench.py --gpus 1 --force-dist --gather-impl torch -- \
 p1 200 python bench.py -- \
 g1 300 $TR --master-port 29514 bench.py --gpus 1 --force-dist -- \
 n1 300 $TR --master-port 29515 bench.py --gpus 1 --force-dist --dist-backend nccl -- \
 t1 300 $TR --master-port 29516 bench.py --gpus 1 --force-dist --gather-impl torch -- \
 p2 200 python bench.py -- \
 g2 300 $TR --master-port 29517 bench.py --gpus 1 --force-dist -- \
 t2 300 $TR --master-port 29518 bench.py --gpus 1 --force-dist --gather-impl torch
