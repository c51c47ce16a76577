import os, sys, time
sys.path.insert(0, "chiaroscuro-raytracer_amd")
os.environ.setdefault("CHIARO_QUIET", "1")
import torch
import chiaroscuro_amd as ca
from chiaroscuro_amd import scenes
from chiaroscuro_amd.tiles import DistributedFrame
cfg = sys.argv[1]; L = int(sys.argv[2])
sc = ca.Scene(scenes.config_rtc(cfg)); i = sc.info; m = ca.Model(sc)
dev = ca.Device(0); dev.upload(ca.KDTree(m, sc).describe()); dev.set_option("counters", 0)
cam = ca.camera(i["VP"], i["LA"], i["UP"], i["yview"], i["xres"], i["yres"])
fr = DistributedFrame(dev, i["xres"], i["yres"], 0, 1, 32)
if len(sys.argv) > 3:  # a full-frame single layer first, as bench.py's warmup
    a = time.perf_counter()
    fr.render_layer(cam, ca.render_params(i["xres"], i["yres"], i["samples"], i["k"], i["seed"], layer=1))
    torch.cuda.synchronize()
    print("warmup layer wall %.1f kernel %.1f ms" % ((time.perf_counter() - a) * 1e3, dev.last_kernel_ms()), flush=True)
for rep in range(2):
    p = ca.render_params(i["xres"], i["yres"], i["samples"], i["k"], i["seed"], layer=2 + rep * L)
    t0 = time.perf_counter(); nl, pieces = fr.plan_layers(p, L); t1 = time.perf_counter()
    q = ca.render_params(i["xres"], i["yres"], i["samples"], i["k"], i["seed"], layer=2 + rep * L)
    walls, ks = [], []
    for k in range(pieces):
        q.rank, q.nranks = k, pieces
        a = time.perf_counter(); dev.render_layers_device(cam, q, nl, fr.frame.data_ptr()); torch.cuda.synchronize(); b = time.perf_counter()
        walls.append((b - a) * 1e3); ks.append(dev.last_kernel_ms())
    print(cfg, L, "plan %.1f ms" % ((t1 - t0) * 1e3), nl, pieces, "wall %.1f kernel %.1f ms" % (sum(walls), sum(ks)),
          "per pass wall-kernel: " + " ".join("%.1f" % (w - k) for w, k in zip(walls, ks))[:300], flush=True)
