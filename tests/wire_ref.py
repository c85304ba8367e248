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
