import ctypes, os, torch, time
lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "libprobe.so"))
x = torch.zeros(1000, device="cuda")
s = torch.cuda.current_stream().cuda_stream
print("rt version", lib.probe_runtime_version())
r = lib.probe_add_one(ctypes.c_void_p(x.data_ptr()), 1000, ctypes.c_void_p(s))
torch.cuda.synchronize()
print("ret", r, "sum", x.sum().item(), torch.cuda.get_device_name(0))
import subprocess
print(open("/proc/self/maps").read().count("libamdhip64"), [l for l in open("/proc/self/maps").read().splitlines() if "libamdhip64" in l][:1])
