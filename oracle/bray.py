"""ORACLE tool (test infrastructure): freeze SURVEY.md §8(d)'s algorithmic bytes per primary ray,
B_ray = 16*E_node + 4*E_child + B_out with E_node = E_child + 1, where E_child counts node entries
along the reference DDA path under the shader's common-ancestor restart (low_res.frag:493-531) on
the reference-format tree.  Writes profiles/bray.json, which bench.py reads (it never imports the
oracle for this).  Usage: python oracle/bray.py [C3f | C2d8 | C3_shade]  (one entry only, merged into the existing file;
C3_shade: the shading pass, see c3_shade_entry)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

B_OUT = 24


C3F_ORIGIN = (4.37, 90.61, 4.23)  # bench.py CONFIGS["c3f"]


def c3f_entry():
    t = O.Tree.terrain(6, 4096, 4096)
    e = t.frame_entries(C3F_ORIGIN, O.normalize((1, -0.45, 1)), 1920, 1080, 16384, nthreads=8) / (1920 * 1080)
    return {"e_child_per_ray": e, "bytes_per_ray": 16 * (e + 1) + 4 * e + B_OUT,
            "tree": "as C3, camera at %s (non-integral: segment-exact crossings)" % (C3F_ORIGIN,)}


def c2d8_entry():
    # BASELINE.json config 2 as worded: depth 8 = a 4-level (256^3) tree, putBlock / genWorld over 200 x 200 columns
    t = O.Tree.terrain_putblock(4, 200, 200)
    e = t.frame_entries((4, 90, 4), O.normalize((1, -0.45, 1)), 1920, 1080, 300, nthreads=8) / (1920 * 1080)
    return {"e_child_per_ray": e, "bytes_per_ray": 16 * (e + 1) + 4 * e + B_OUT,
            "tree": "depth-8 (4 levels, 256^3): clean root + genWorld putBlocks over 200 x 200 columns; C3 pose, S = 300"}


SUN = (2.0, 1.0, 4.0)  # the reference sun (globals.cpp:23), normalised as rt.sun_dir() does


def c3_shade_entry():
    """bench.py --shade: the shading pass over the C3 frame with water (liquid mode), S = 16384, 75-step shadow rays.
    B_ray = 16 (E + R) + 4 E + 16: E node entries per pixel under the restart model (primary with its reflections /
    refractions, plus the shadow ray continuing from the primary's lookup state), R root reads per pixel (the primary
    and, where one is cast, the shadow ray), and the 16-B rgba pixel (the bench writes no hit records)."""
    t = O.Tree.terrain(6, 4096, 4096)
    n = 1920 * 1080
    e, sh, lk = t.shade_entries((4, 90, 4), O.normalize((1, -0.45, 1)), 1920, 1080, 16384, O.normalize(SUN), 75, nthreads=8,
                                liquid=True)
    E, R = e / n, 1.0 + sh / n
    return {"e_per_ray": E, "shadow_rays_per_ray": sh / n, "lookups_per_ray": lk / n, "bytes_per_ray": 16 * (E + R) + 4 * E + 16,
            "formula": "16 (E + R) + 4 E + 16 B rgba, R = 1 + shadow rays per pixel",
            "tree": "depth-12 terrain (4096^2 columns), reference node/array format, liquid mode (water refracts); C3 pose, S = 16384, "
                    "sun normalize(2,1,4), 75-step shadow rays"}


def main():
    if sys.argv[1:] == ["C3_shade"]:
        path = os.path.join(ROOT, "profiles", "bray.json")
        res = json.load(open(path))
        res["C3_shade"] = c3_shade_entry()
        json.dump(res, open(path, "w"), indent=1)
        print(json.dumps(res["C3_shade"], indent=1))
        return
    if sys.argv[1:] == ["C2d8"]:
        path = os.path.join(ROOT, "profiles", "bray.json")
        res = json.load(open(path))
        res["C2d8"] = c2d8_entry()
        json.dump(res, open(path, "w"), indent=1)
        print(json.dumps(res["C2d8"], indent=1))
        return
    if sys.argv[1:] == ["C3f"]:
        path = os.path.join(ROOT, "profiles", "bray.json")
        res = json.load(open(path))
        res["C3f"] = c3f_entry()
        json.dump(res, open(path, "w"), indent=1)
        print(json.dumps(res["C3f"], indent=1))
        return
    res = {"formula": "B_ray = 16*(E_child+1) + 4*E_child + B_out, B_out = %d (this build's hit record)" % B_OUT,
           "source": "oracle/bray.py (orc_frame_entries, oracle/oracle.c)"}
    ref = O.Tree.reference_world()
    for name, org, d, s in (("C2_cam0_S300", (35, 50, 35), (1, 0, 1), 300), ("C2_cam1_S300", (4, 90, 4), (1, -0.45, 1), 300),
                            ("C2_cam1_S600", (4, 90, 4), (1, -0.45, 1), 600)):
        e = ref.frame_entries(org, O.normalize(d), 1920, 1080, s, nthreads=8) / (1920 * 1080)
        res[name] = {"e_child_per_ray": e, "bytes_per_ray": 16 * (e + 1) + 4 * e + B_OUT, "tree": "reference world (putBlock)"}
    t = O.Tree.terrain(6, 4096, 4096)
    e = t.frame_entries((4, 90, 4), O.normalize((1, -0.45, 1)), 1920, 1080, 16384, nthreads=8) / (1920 * 1080)
    res["C3"] = {"e_child_per_ray": e, "bytes_per_ray": 16 * (e + 1) + 4 * e + B_OUT,
                 "tree": "depth-12 terrain, reference node/array format with uniform regions collapsed"}
    res["C3f"] = c3f_entry()
    res["C2d8"] = c2d8_entry()
    res["C3_shade"] = c3_shade_entry()
    # C4: §8(d) "for AO: add <= 5 steps x E per sample" -- the AO rays' node entries (each continues the
    # restart model from the primary's final lookup), 16 + 4 B per entry, per primary ray of the frame;
    # B_OUT grows by the 1-B AO count
    for n_ao in (16, 20):
        ea = t.frame_entries_ao((4, 90, 4), O.normalize((1, -0.45, 1)), 1920, 1080, 16384, n_ao, 5, nthreads=8) / (1920 * 1080)
        res["C4_ao%d" % n_ao] = {"e_child_per_ray": e, "e_ao_per_ray": ea,
                                 "bytes_per_ray": 16 * (e + 1) + 4 * e + 20 * ea + B_OUT + 1,
                                 "tree": "as C3; AO %d samples x 5 steps per hit" % n_ao}
    # C5: 7 levels, 3840x2160 from the same pose; every ray lands within ~2,600 voxels of the camera,
    # so the oracle tree over the first 4096^2 columns of the 16384^2 terrain sees exactly the same
    # voxels (a full 16384^2 reference-format tree would exceed the 2^32-byte pools)
    t = O.Tree.terrain(7, 4096, 4096)
    e = t.frame_entries((4, 90, 4), O.normalize((1, -0.45, 1)), 3840, 2160, 16384, nthreads=8) / (3840 * 2160)
    res["C5"] = {"e_child_per_ray": e, "bytes_per_ray": 16 * (e + 1) + 4 * e + B_OUT,
                 "tree": "depth-14 (7 levels), first 4096^2 columns, reference node/array format, uniform regions collapsed"}
    # C1: the dense 256^3 grid, "1 B per DDA step plus output" (§8d), reference camera, 256^2 rays, S = 300
    D = O.Dense(ref, 256)
    r = D.cast_frame((35, 50, 35), O.normalize((1, 0, 1)), 256, 256, 300)
    st = r["dda_steps"] / (256 * 256)
    res["C1"] = {"dda_steps_per_ray": st, "bytes_per_ray": st + B_OUT, "tree": "dense u8 grid of the reference world's [0,256)^3"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "profiles", "bray.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
