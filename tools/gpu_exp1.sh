#!/bin/bash
# Experiments: baseline vs cluster-sorted queries vs f16 storage; 2-rank gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "base:" "sorted:--sort-queries cluster" "f16:--quant f16" "f16sorted:--quant f16 --sort-queries cluster"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --no-cpu --steps 5 $args > gpurun_out/exp_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/exp_$tag.log; exit $rc; }
  python -c "import json;d=json.loads(open('gpurun_out/exp_$tag.log').read().strip().splitlines()[-1]);print('$tag', d['value'], d['config']['ef'], d['config']['recall_at_10'], d['roofline']['kernel_ms'], d['build_vectors_per_s'])"
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --rows 200000 --queries 2000 --gt-queries 500 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -1 gpurun_out/bench_gloo2.log
exit $rc
