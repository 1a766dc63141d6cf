import ctypes as C, sys, os, time
import torch
torch.cuda.set_device(0)
x = torch.ones(4, device='cuda'); print('torch ok', x.sum().item())
sys.path.insert(0, 'bevy-hikari_amd')
import hikari_amd
L = hikari_amd._abi.lib()
with open('/proc/self/maps') as f:
    print(sorted(set(l.split()[-1] for l in f if 'amdhip' in l or 'hsa-runtime' in l)))
from hikari_amd import HikariRenderer, HikariSettings, Upscale, examples, frame_inputs
scene, cam, lights = examples.cornell(); scene.build()
W, H = 1920, 1080
st = HikariSettings(upscale=Upscale.SMAA_TU_1_0, indirect_spatial_reuse=False, denoise=False); s = st.to_c()
r = HikariRenderer(0); r.set_noise(); r.upload_scene(scene); r.resize(W, H, 1.0)
sp = torch.cuda.current_stream().cuda_stream
for f in range(30):
    fi = frame_inputs(f, cam, lights, W, H); r.render_gbuffer(fi, sp); r.render_frame(s, fi, sp); r.tone_sum(s, sp)
torch.cuda.synchronize(); t = time.time()
for f in range(30, 80):
    fi = frame_inputs(f, cam, lights, W, H); r.render_gbuffer(fi, sp); r.render_frame(s, fi, sp); r.tone_sum(s, sp)
torch.cuda.synchronize(); print('ms/frame', (time.time() - t) / 50 * 1e3)
t = torch.empty((H, W, 4), dtype=torch.float16, device='cuda')
r.copy_output_rows(10, 0, H, t.data_ptr(), False, sp); torch.cuda.synchronize()
print('tone mean', t.float()[..., :3].mean().item())
os.environ.setdefault('MASTER_ADDR', '127.0.0.1'); os.environ.setdefault('MASTER_PORT', '29555')
import torch.distributed as dist
dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
full = torch.empty_like(t); dist.all_gather_into_tensor(full, t); torch.cuda.synchronize()
print('allgather ok', torch.equal(full, t)); dist.destroy_process_group()
