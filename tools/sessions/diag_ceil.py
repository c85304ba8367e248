import sys, numpy as np
sys.path.insert(0, '.')
import raytracing_test_amd as rt
from oracle import oracle as O
w = rt.World.reference()
t = w.build().upload(0)
cams = [((35.0, 50.0, 35.0), (1.0, 0.0, 1.0)), ((4.0, 90.0, 4.0), (1.0, -0.45, 1.0)), ((100.0, 120.0, 100.0), (1.0, -1.2, 0.3)),
        ((150.3, 44.7, 20.9), (-0.6, -0.2, 1.0))]
T = O.Tree.reference_world()
for org, d in cams:
    dn = rt.normalize(d)
    for S in (30, 300):
        a = rt.decode_hits(t.cast_frame(org, dn, 64, 48, S))
        b = rt.decode_hits(t.cast_frame(org, dn, 64, 48, S, flags=rt.CAST_NO_CEILINGS))
        ref = T.cast_frame(org, dn, 64, 48, S)
        bad = np.nonzero((a["pos"] != ref["pos"]).any(1) | (a["steps"] != ref["steps"]))[0]
        badb = np.nonzero((b["pos"] != ref["pos"]).any(1))[0]
        print(org, S, "ceil mismatches", len(bad), "noceil mismatches", len(badb))
        for i in bad[:3]:
            print("  pix", i, "gpu", a["pos"][i], a["steps"][i], a["hit"][i], "ref", ref["pos"][i], ref["steps"][i], ref["hit"][i], "noceil", b["pos"][i], b["steps"][i])
c = t.ceilings()
print("ceil64 block(0,0..3)", c[0][0, :4], "max", c[0].max(), c[1].max())
# edits as the bridge test makes them, then a frame
from oracle import oracle as O2
T2 = O2.Tree.reference_world()
w2 = rt.World.reference()
t2 = w2.build().upload(0)
for (x, y, z, lvl, put) in ((20, 80, 20, 5, True), (20, 80, 20, 5, False), (41, 40, 58, 6, False)):
    if put:
        w2.put_block(x, y, z, 0, 777, 0.0, lvl); T2.put_block(x, y, z, 0, 777, 0.0, lvl)
    else:
        w2.delete_block(x, y, z, lvl); T2.delete_block(x, y, z, level=lvl)
    t2.update(w2, np.array([[x, y, z]], np.int32), level=lvl)
    t2.sync()
for org, d in cams:
    dn = rt.normalize(d)
    a = rt.decode_hits(t2.cast_frame(org, dn, 64, 48, 300))
    b = rt.decode_hits(t2.cast_frame(org, dn, 64, 48, 300, flags=rt.CAST_NO_CEILINGS))
    ref = T2.cast_frame(org, dn, 64, 48, 300)
    print("edited", org, "ceil mismatches", int(((a["pos"] != ref["pos"]).any(1)).sum()), "noceil", int(((b["pos"] != ref["pos"]).any(1)).sum()))
