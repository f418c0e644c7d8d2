#!/bin/bash
# Same-box A/B of the LayerNorm backward grid (MSQ_LNB_BLOCKS) and its dx_acc prefetch (MSQ_LNB_PF).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/ab_$tag.json 2>gpurun_out/ab.err || return 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));c=d['classes'];print('$tag', d['ms_per_step'], 'lnb', c['other:layernorm_bwd_bias']['ms_per_step'])"
}
run b512 A=1 && run b768 MSQ_LNB_BLOCKS=768 && run b1024 MSQ_LNB_BLOCKS=1024 && run b768pf MSQ_LNB_BLOCKS=768 MSQ_LNB_PF=1 && run b1024pf MSQ_LNB_BLOCKS=1024 MSQ_LNB_PF=1 && run b512_2 A=1 && run b768_2 MSQ_LNB_BLOCKS=768 && run b1024_2 MSQ_LNB_BLOCKS=1024
