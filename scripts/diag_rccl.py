"""Diagnose the native RCCL communicator on one GPU (world 1)."""
import os, sys, faulthandler
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
mode = sys.argv[1] if len(sys.argv) > 1 else "native"
torch.cuda.set_device(0)
x = torch.ones(1024, device="cuda")
if mode == "torch":
    import torch.distributed as dist
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29641", rank=0, world_size=1)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print("torch nccl ok", float(x[0]))
else:
    from torch_distlearn_amd import _native
    C = _native.native()
    print("rccl version", C.rccl_version(), flush=True)
    uid = C.rccl_unique_id()
    print("uid ok", len(uid), flush=True)
    c = C.RcclCommunicator(uid, 0, 1, 0)
    print("comm ok", flush=True)
    c.all_reduce(x.data_ptr(), x.data_ptr(), x.numel(), 0, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print("native allreduce ok", float(x[0]))
