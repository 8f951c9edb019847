import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hyper-ray-tracer_amd"))
import numpy as np, torch, hrt
s = hrt.preset("random", 1); s.commit(0)
cam = hrt.preset_camera(s.info, 64, 36)
p = hrt.params(64, 36, 8, 3, 11, tuple(s.info.background))
full, st = hrt.render(s, cam, p, stats=True)
print("full", st.pixels, st.samples, st.segments)
for reg in [(0,0,64,36),(0,0,20,17),(10,0,20,17),(0,5,20,17),(10,5,20,17),(8,8,16,16),(10,5,24,24)]:
    part, st = hrt.render(s, cam, p, region=reg, stats=True)
    x0,y0,w,h = reg
    ok = np.array_equal(full[y0:y0+h, x0:x0+w], part)
    print(reg, "pixels", st.pixels, "samples", st.samples, "seg", st.segments, "equal", ok, "max|part|", float(np.nanmax(np.abs(part))))
    d = torch.full((h, w, 4), -7.0, device="cuda")
    st2 = hrt.render_tiles_device(s, cam, p, [reg], d.data_ptr(), 0, want_stats=True)
    torch.cuda.synchronize()
    dd = d.cpu().numpy()
    print("   device-path pixels", st2.pixels, "equal", np.array_equal(dd, full[y0:y0+h, x0:x0+w]), "unwritten", int((dd[...,3] == -7).sum()))
