"""hipMalloc time against size on one MI355X (round 6: a chunk's path state above ~160 GB took seconds
to allocate). Allocates and frees one buffer of each size through librtg's runtime (torch's
allocator calls hipMalloc for blocks this big), and prints JSON lines."""
import json
import time

import torch

free, total = torch.cuda.mem_get_info()
print(json.dumps({"free_gb": free / 2**30, "total_gb": total / 2**30}), flush=True)
for gb in (32, 96, 128, 144, 152, 160, 168, 176, 184, 192):
    if gb * 2**30 > free * 0.9:
        break
    torch.cuda.synchronize()
    t = time.time()
    x = torch.empty(gb * 2**30, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ta = time.time() - t
    t = time.time()
    x[::2**20] = 1  # touch one byte per MiB
    torch.cuda.synchronize()
    tt = time.time() - t
    del x
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    print(json.dumps({"gb": gb, "alloc_s": round(ta, 3), "touch_s": round(tt, 3)}), flush=True)
