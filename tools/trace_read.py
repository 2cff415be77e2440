import numpy as np, sys, os, time
sys.path.insert(0, os.getcwd())
import lstore_amd as L
k, m, C, N = 6, 3, 65536, 1000
data = np.random.default_rng(0).integers(0, 256, (N, k, C), dtype=np.uint8)
p = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
img = p.segment_write(data, 1, 0)
deg = img.copy(); deg[0].reshape(N, C + 4)[:, 0] ^= 0x11
for name, im, par in (("paranoid", img, True), ("degraded", deg, False)):
    for rep in range(3):
        t0 = time.perf_counter(); out, st, bad = p.segment_read(im, N, C, 1, 0, paranoid=par); t = time.perf_counter() - t0
        print(name, rep, round(t * 1e3, 2), "ms", flush=True)
