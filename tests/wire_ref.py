"""numpy restatement of the 12-B hit-record wire format (include/svo_rt.h, svo_hits_pack /
svo_hits_unpack) — test infrastructure: the GPU kernels are checked against it, and the CPU gloo
test gathers records in this format."""
import numpy as np

HIT_BIT, AXIS_SHIFT, NEG_BIT = 1 << 31, 16, 1 << 18


def pack(pos_steps, t, info, cells):
    """records (n,4) i32, (n,) f32, (n,) u32 + origin cells (n,3) i32 -> (n, 12) uint8"""
    info = info.astype(np.uint32)
    d = (pos_steps[:, :3].astype(np.int64) - cells).astype(np.int16)
    i16 = ((info >> 31) << 15) | (((info >> AXIS_SHIFT) & 3) << 13) | (((info & NEG_BIT) != 0).astype(np.uint32) << 12) | (info & 0xFFF)
    rec = np.zeros((len(t), 6), np.uint16)
    rec[:, 0:3] = d.view(np.uint16)
    rec[:, 3] = i16.astype(np.uint16)
    rec[:, 4:6] = np.ascontiguousarray(t.astype(np.float32)).view(np.uint16).reshape(-1, 2)
    return rec.view(np.uint8).reshape(-1, 12)


def unpack(wire, cells, steps):
    rec = np.ascontiguousarray(wire).view(np.uint16).reshape(-1, 6)
    d = rec[:, 0:3].view(np.int16).astype(np.int32)
    i16 = rec[:, 3].astype(np.uint32)
    hit = (i16 >> 15) != 0
    left = np.where(hit, steps - np.abs(d).sum(1), 0).astype(np.int32)
    pos_steps = np.concatenate([cells + d, left[:, None]], 1).astype(np.int32)
    info = (hit.astype(np.uint32) << 31) | (((i16 >> 13) & 3) << AXIS_SHIFT) | (((i16 >> 12) & 1) << 18) | (i16 & 0xFFF)
    t = np.ascontiguousarray(rec[:, 4:6]).view(np.float32).reshape(-1)
    return pos_steps, t, info.astype(np.uint32)


# ---- the 8-B compact records (frames from integral / half-integral camera positions) ----
def pack_compact(pos_steps, info, cells):
    """records + origin cells -> (n, 8) uint8: n_x | n_y << 15 | n_z << 30 | hit << 45 | axis << 46 | material << 48"""
    info = info.astype(np.uint64)
    nk = np.abs(pos_steps[:, :3].astype(np.int64) - cells).astype(np.uint64)
    rec = nk[:, 0] | (nk[:, 1] << np.uint64(15)) | (nk[:, 2] << np.uint64(30)) | ((info >> np.uint64(31)) << np.uint64(45)) | \
        (((info >> np.uint64(AXIS_SHIFT)) & np.uint64(3)) << np.uint64(46)) | ((info & np.uint64(0xFFF)) << np.uint64(48))
    return np.ascontiguousarray(rec.astype(np.uint64)).view(np.uint8).reshape(-1, 8)


def unpack_compact(wire, origins, dirs, steps):
    """(n, 8) records + each record's ray (origin, direction: float32) -> (pos_steps, t, info): the ray is
    rebuilt as castRayFromCam's buildRay (src/ray_caster.cpp:19-44) and its deltaPos after n steps on the
    last axis is T0 + n a (exact sums from such origins), t the crossing before it"""
    rec = np.ascontiguousarray(wire).view(np.uint64).reshape(-1)
    nk = np.stack([(rec >> np.uint64(15 * k)) & np.uint64(0x7FFF) for k in range(3)], 1).astype(np.int64)
    hit = ((rec >> np.uint64(45)) & np.uint64(1)) != 0
    axis = ((rec >> np.uint64(46)) & np.uint64(3)).astype(np.int64)
    mat = ((rec >> np.uint64(48)) & np.uint64(0xFFF)).astype(np.uint32)
    o = origins.astype(np.float32)
    d = dirs.astype(np.float32)
    step = np.where(d < 0, -1, 1)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        delta = (np.float32(1.0) / d).astype(np.float64)
        ad = np.abs(delta)
        cell = np.trunc(o).astype(np.int64)
        exact = o.astype(np.float64) - np.where(step < 0, 1.0, 0.0)
        T0 = ad - (exact - cell) * delta
        pos = cell + step * nk
        rows = np.arange(len(rec))
        ax = np.minimum(axis, 2)
        T = nk[rows, ax] * ad[rows, ax] + T0[rows, ax]
        t = np.where(np.isinf(ad[rows, ax]), T, T - ad[rows, ax])
    t = np.where(axis == 3, 0.0, t).astype(np.float32)
    neg = (axis < 3) & (step[rows, ax] < 0)
    left = np.where(hit, steps - nk.sum(1), 0)
    info = (hit.astype(np.uint32) << 31) | (axis.astype(np.uint32) << AXIS_SHIFT) | (neg.astype(np.uint32) << 18) | mat
    return np.concatenate([pos, left[:, None]], 1).astype(np.int32), t, info.astype(np.uint32)
