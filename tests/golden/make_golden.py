"""Regenerate the golden vectors in tests/golden/ from the REFERENCE itself (run in the build
container, where /root/reference exists; the GPU box only reads the committed outputs).

Sources (all reference-produced, none from this repo's code):
  * noise_ref.npz     — include/OpenSimplexNoise.cpp compiled from /root/reference by oracle/Makefile
                        (oracle/_ref/libref_noise.so): Noise(seed).eval(x, y) at world-gen sample
                        points and random points, seeds 42/64/100 (world_gen.cpp:15-17) + others.
  * hemisphere_ref.json — stdout of /root/reference/gen_hemisphare_distrib.py (N = 20, run with
                        MPLBACKEND=Agg), plus the 20 literals of src/shaders/light_scattering.frag:
                        134-153 as DATA (the float32 table the shader uses).
  * reference_facts.json — values the survey recorded by compiling and running the reference's own
                        C++: test.cpp's known answer, the reference world's
                        node / array counts, root bitmap, wrap and max-depth behaviour, the pick ray
                        and the frame statistics at the default camera.
"""
import json
import os
import re
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)


def noise():
    from oracle import oracle as O

    O.build_ref()
    rng = np.random.default_rng(20250620)
    xs, ys, seeds = [], [], []
    for seed in (42, 64, 100, 0, 1, -5, 987654321987):
        for scale in (0.005, 0.05, 0.1):
            gx = rng.integers(0, 16384, 300)
            gz = rng.integers(0, 16384, 300)
            xs.append(gx * scale)
            ys.append(gz * scale)
            seeds.append(np.full(300, seed))
        xs.append(rng.uniform(-2000, 2000, 500))
        ys.append(rng.uniform(-2000, 2000, 500))
        seeds.append(np.full(500, seed))
    x = np.concatenate(xs)
    y = np.concatenate(ys)
    s = np.concatenate(seeds).astype(np.int64)
    v = np.zeros_like(x)
    for seed in np.unique(s):
        m = s == seed
        v[m] = O.ref_noise_batch(int(seed), x[m], y[m])
    np.savez_compressed(os.path.join(HERE, "noise_ref.npz"), x=x, y=y, seed=s, value=v)


def hemisphere():
    env = dict(os.environ, MPLBACKEND="Agg")
    out = subprocess.run([sys.executable, os.path.join(REF, "gen_hemisphare_distrib.py")], capture_output=True, text=True,
                         env=env, cwd="/tmp", timeout=300, check=True).stdout
    py = [[float(a) for a in m] for m in re.findall(r"vec3\(([^,]+),([^,]+),([^)]+)\)", out)]
    frag = open(os.path.join(REF, "src/shaders/light_scattering.frag")).read()
    block = frag[frag.index("vec3[] hemisphereDirs"):]
    block = block[: block.index("};")]
    lit = [[float(a) for a in m] for m in re.findall(r"vec3\(([^,]+),([^,]+),([^)]+)\)", block)]
    json.dump({"source": "gen_hemisphare_distrib.py stdout (x, z, y order as printed) and light_scattering.frag:134-153",
               "n": 20, "polar_span": 0.85, "generator_stdout": py, "shader_literals": lit},
              open(os.path.join(HERE, "hemisphere_ref.json"), "w"), indent=1)


def facts():
    f = {
        "provenance": "SURVEY.md probes: the reference C++ (tetrahexa_tree.cpp, voxel_allocator.cpp, world_gen.cpp, "
                      "ray_caster.cpp, OpenSimplexNoise.cpp, test.cpp) compiled and run in the survey container",
        "test_cpp_kat": {"dir_unnormalized": [11, 20, 3], "origin": [10.5, 12.1, 14.7], "steps": 500,
                         "last_hit": 1, "round": [172, 306, 58], "source": "SURVEY.md §4 (test.cpp:78-134)"},
        "reference_world": {"nodes": 1172118, "arrays": 20724, "root_bitmap": "0x8000000000000001",
                            "source": "SURVEY.md §0.2, §3A, §6"},
        "wrap": {"a": [1034, 5, 10], "b": [10, 5, 10], "equal": True, "source": "SURVEY.md §8a A2"},
        "max_depth_exit": {"points": [[778, 773, 778], [960, 960, 960]], "source": "SURVEY.md §0.2"},
        "debug_blocks": {"level5_leaf": {"min": [20, 8, 200], "max": [23, 11, 203], "flags": 5},
                         "reflective_voxel": {"pos": [10, 100, 10], "flags": 3}, "source": "SURVEY.md §8a A2"},
        "pick_ray_default_camera": {"origin": [35, 50, 35], "dir_unnormalized": [1, 0, 1],
                                    "walks_axis": 2, "source": "SURVEY.md §0.3"},
        "frame_default_camera": {"width": 1920, "height": 1080, "steps": 300, "hit_fraction": 0.469,
                                 "mean_dda_steps": 169.8, "tolerance": [0.0005, 0.05], "source": "SURVEY.md §6"},
        "terrain_4096_height_range": {"min": 1, "max": 63, "source": "SURVEY.md §7 (hard parts: scale)"},
    }
    json.dump(f, open(os.path.join(HERE, "reference_facts.json"), "w"), indent=1)


if __name__ == "__main__":
    noise()
    hemisphere()
    facts()
    print("golden vectors written to", HERE)
