import ctypes as C, sys, os
sys.path.insert(0, 'bevy-hikari_amd')
import hikari_amd
L = hikari_amd._abi.lib()
hip = C.CDLL('libamdhip64.so.7')
n = C.c_int(-1); rc = hip.hipGetDeviceCount(C.byref(n)); print('before torch: count rc', rc, n.value)
h = C.c_void_p(); print('hk_create before torch', L.hk_create(0, C.byref(h)), L.hk_last_error(None))
if h.value: L.hk_destroy(h)
import torch
print('torch', torch.__version__, torch.cuda.is_available())
torch.cuda.set_device(0)
n = C.c_int(-1); rc = hip.hipGetDeviceCount(C.byref(n)); print('after torch: count rc', rc, n.value)
h = C.c_void_p(); print('hk_create after torch', L.hk_create(0, C.byref(h)))
with open('/proc/self/maps') as f:
    print(sorted(set(l.split()[-1] for l in f if 'amdhip' in l or 'hsa-runtime' in l)))
