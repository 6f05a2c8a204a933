import ctypes, os, torch
assert torch.cuda.is_available()
x = torch.arange(1000, device='cuda', dtype=torch.float32) + 0.5
lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), 'libprobe.so'))
s = torch.cuda.current_stream().cuda_stream
err = lib.probe_launch(ctypes.c_void_p(x.data_ptr()), ctypes.c_int(1000), ctypes.c_void_p(s))
torch.cuda.synchronize()
print('err', err, x[:6].tolist())
maps = open('/proc/self/maps').read()
print('amdhip mapped:', sorted(set(l.split()[-1] for l in maps.splitlines() if 'amdhip64' in l)))
print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).gcnArchName)
import subprocess; print(subprocess.run(['lscpu'],capture_output=True,text=True).stdout[:800])
print('cpu cap', torch.backends.cpu.get_cpu_capability(), os.cpu_count())
