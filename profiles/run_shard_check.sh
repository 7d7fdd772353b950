# pair-granular frame shard on the GPU box: the 2-rank HIP shard test, the
# default bench line, and 2-rank gloo rehearsals (one GPU) of c2 and cut c5
set -o pipefail
O=gpurun_out/shard; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_shard.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
VAME_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 2 > $O/c2_gloo2.json 2> $O/c2_gloo2.err || exit 1
VAME_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --config c5 --frames 24 --steps 2 --warmup 1 > $O/c5_gloo2.json 2> $O/c5_gloo2.err || exit 1
python -c "
import json
for c in ('bench_default','c2_gloo2','c5_gloo2'):
    d=json.loads([l for l in open('$O/%s.json'%c) if l.startswith('{')][-1]); print(c, d['ms_per_step'], d['value']/1e6, d['config']['pairs_per_step_rank0'], d['gather']['check'])
"
