# interleaved A/B of the multi-rank bench path on one GPU:
# p = plain bench.py; n = torchrun 1 rank --force-dist, native RCCL gather; t = same with torch.distributed.gather
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
bash tools/gpu_session.sh \
 p0 200 python bench.py -- \
 n0 300 $TR --master-port 29511 bench.py --gpus 1 --force-dist -- \
 t0 300 $TR --master-port 29512 bench.py --gpus 1 --force-dist --gather-impl torch -- \
 p1 200 python bench.py -- \
 n1 300 $TR --master-port 29513 bench.py --gpus 1 --force-dist -- \
 t1 300 $TR --master-port 29514 bench.py --gpus 1 --force-dist --gather-impl torch -- \
 p2 200 python bench.py -- \
 n2 300 $TR --master-port 29515 bench.py --gpus 1 --force-dist -- \
 t2 300 $TR --master-port 29516 bench.py --gpus 1 --force-dist --gather-impl torch
