"""Does this PyTorch-ROCm build honour expandable segments?  Allocate 3 x 8 GiB, free the
middle one, allocate 12 GiB: a segmented cache needs a new 12 GiB segment (reserved 28 GiB);
expandable segments grow one mapping (reserved ~28 too, but device allocs differ) -- the
snapshot's segment types say which allocator ran."""
import os
import sys
import torch

how = sys.argv[1] if len(sys.argv) > 1 else "env"
if how == "api":
    torch.cuda.memory._set_allocator_settings("expandable_segments:True")
G = 2 ** 30
a = torch.empty(8 * G, dtype=torch.uint8, device="cuda")
b = torch.empty(8 * G, dtype=torch.uint8, device="cuda")
c = torch.empty(8 * G, dtype=torch.uint8, device="cuda")
del b
d = torch.empty(12 * G, dtype=torch.uint8, device="cuda")
ms = torch.cuda.memory_stats()
snap = torch.cuda.memory_snapshot()
print(how, os.environ.get("PYTORCH_HIP_ALLOC_CONF"), os.environ.get("PYTORCH_CUDA_ALLOC_CONF"),
      "reserved GiB", ms["reserved_bytes.all.current"] / G, "device allocs", ms["num_device_alloc"],
      "segments", len(snap), "types", sorted({str(s.get("segment_type")) + "/" + str(s.get("is_expandable")) for s in snap}),
      flush=True)
