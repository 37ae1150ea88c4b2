import os, torch, torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
import torch.distributed._symmetric_memory as symm
try:
    t = symm.empty(1024, dtype=torch.float32, device="cuda:0")
    hdl = symm.rendezvous(t, dist.group.WORLD.group_name)
    t.fill_(2.0)
    out = torch.ops.symm_mem.one_shot_all_reduce(t, "sum", dist.group.WORLD.group_name)
    torch.cuda.synchronize()
    print("one_shot ok", float(out[0]), out.shape)
except Exception as e:
    print("symm ERR", type(e).__name__, str(e)[:300])
dist.destroy_process_group()
