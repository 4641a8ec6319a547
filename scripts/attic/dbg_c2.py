"""Debug: run test_mbconv_fused_middle_vs_fp32_torch with every rel() printed."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd"), os.path.join(ROOT, "tests")]
import test_c2_bf16_gpu as m
orig = m.rel
def rel(a, b):
    v = orig(a, b)
    print(f"  rel {v:.5f}  shapes {tuple(a.shape)}", flush=True)
    return v
m.rel = rel
for args in [(4, 19, 64, 2), (4, 19, 64, 1), (3, 30, 32, 2)]:
    print(args, flush=True)
    try:
        m.test_mbconv_fused_middle_vs_fp32_torch(*args)
        print("  PASS", flush=True)
    except AssertionError as e:
        print("  FAIL", str(e)[:100], flush=True)
