"""Step-by-step bring-up diagnostic (prints progress; faulthandler on)."""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def p(*a):
    print(*a, flush=True)


p("import torch")
import torch  # noqa: E402
p("torch", torch.__version__, torch.version.hip, "avail", torch.cuda.is_available())
p("dev0", torch.cuda.get_device_name(0))
x = torch.ones(4, device="cuda:0")
p("torch tensor ok", float(x.sum()))
p("import ciruela_amd")
import ciruela_amd as ca  # noqa: E402
p("maps:", sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip" in l or "hsa-runtime" in l}))
p("device_count", ca._n.lib.cir_device_count())
ctx = ca.Context(device_mask=1)
p("ctx devices", ctx.devices())
t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda:0")
ca._n.check(ca._n.lib.cir_fill_splitmix64_dev(t.data_ptr(), t.numel(), 1, 0, 0, 0))
torch.cuda.synchronize()
p("fill ok", t[:8].tolist())
out = torch.zeros(32 * 32, dtype=torch.uint8, device="cuda:0")
ctx.hash_chunks_dev(t.data_ptr(), t.numel(), 32768, out.data_ptr(), 0)
torch.cuda.synchronize()
p("chunks ok", out[:32].cpu().numpy().tobytes().hex())
p("hash_bytes abc", ca.BlockHash.hash_bytes(b"abc"))
