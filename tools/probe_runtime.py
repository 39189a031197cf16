"""Probe: a hipcc-built C-ABI .so called through ctypes on torch's current stream."""
import ctypes, subprocess, os, sys
import torch
here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "probe_runtime.so")
subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                       os.path.join(here, "probe_runtime.hip"), "-o", so])
x = torch.randn(64, device="cuda")
ref = torch.exp(x)
lib = ctypes.CDLL(so)
s = torch.cuda.current_stream().cuda_stream
rc = lib.launch(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
print("rc", rc, "maxerr", (x - ref).abs().max().item())
print([l.split()[-1] for l in open('/proc/self/maps') if 'amdhip' in l][:1])
p = torch.cuda.get_device_properties(0)
print(p.name, p.multi_processor_count, p.total_memory/2**30, getattr(p, 'gcnArchName', ''))
print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
