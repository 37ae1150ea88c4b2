# round-5 batch 32: split-K workgroup target A/B on the BERT query pass
set -o pipefail
mkdir -p gpurun_out/r5b32
export TMPDIR=/tmp
O=gpurun_out/r5b32
for t in 512 384 512 384 512 384; do
  AVMI_SPLITK_TARGET=$t timeout -k 10 300 python -u -c "
import json, sys, time, torch
sys.path.insert(0, '.')
from avenir_amd.nn.bert import BertConfig, BertEncoder
torch.manual_seed(0)
m = BertEncoder(BertConfig()).cuda()
ids = torch.randint(0, 30522, (1, 128))
mask = torch.ones_like(ids)
for _ in range(5): m(ids, mask)
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(50): m(ids, mask)
torch.cuda.synchronize()
print(json.dumps({'target': $t, 'ms': (time.perf_counter() - t0) / 50 * 1e3}))
" >> $O/ab.jsonl 2>> $O/ab.err || exit $?
done
