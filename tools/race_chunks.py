#!/usr/bin/env python3
"""Offline attribution of the split contact step's wrong observation float4s
(diagnostics; the dump of tools/contact_race.py with RACE_DUMP).

write_obs_t streams a 64-env workgroup's rows in 8 passes of 8 envs; each pass
copies the blue block (8 envs x 4 rows x 17 float4) and then the red block out
of the LDS stage: flat chunk i of a side's block leaves through store u = i // 64
from lane i % 64. For every wrong float4 of a dumped block this script finds
which correct float4s of the same step and workgroup hold the same 16 bytes,
and tabulates the relation of the best-explaining source to the wrong chunk:
  same pass, other side, same i   (the other side's copy into the same registers)
  next pass, same side, same i    (the next pass's copy)
  previous pass, same side, same i
  next pass, row built by lane i % 64 (the next pass's row build in registers)
  zeros
usage: python tools/race_chunks.py gpurun_out/race_dump.npz"""
import collections
import sys

import numpy as np

EPG, NS, C4 = 8, 4, 17  # envs per pass, rows per side, float4 chunks per row


def block(x, p, side):
    """[EPG*NS*C4, 4] float4 chunks (as int32 bits) of pass p, one side."""
    rows = x[EPG * p:EPG * (p + 1), NS * side:NS * (side + 1)]  # [8, 4, 68]
    return rows.reshape(EPG * NS * C4, 4).view(np.int32)


def main(path):
    d = np.load(path)
    got, want, key = d["got"], d["want"], d["key"]
    rel = collections.Counter()
    by_u = collections.Counter()
    by_lane = collections.Counter()
    n_bad = 0
    for b in range(len(key)):
        g, w = got[b], want[b]
        for p in range(64 // EPG):
            for side in (0, 1):
                gb, wb = block(g, p, side), block(w, p, side)
                bad = np.nonzero((gb != wb).any(1))[0]
                for i in bad:
                    n_bad += 1
                    by_u[(side, i // 64)] += 1
                    by_lane[i % 64 // 16] += 1
                    v = gb[i]
                    hits = []
                    if not v.any():
                        hits.append("zeros")
                    if (block(w, p, 1 - side)[i] == v).all():
                        hits.append("same pass, other side, same i")
                    if p + 1 < 64 // EPG and (block(w, p + 1, side)[i] == v).all():
                        hits.append("next pass, same side, same i")
                    if p > 0 and (block(w, p - 1, side)[i] == v).all():
                        hits.append("previous pass, same side, same i")
                    if p + 1 < 64 // EPG:
                        lane = i % 64
                        e, a = EPG * (p + 1) + lane // 8, lane % 8
                        row = w[e, a].reshape(C4, 4).view(np.int32)
                        if (row == v).all(1).any():
                            hits.append("next pass, row of lane i%64")
                    # anywhere in the step's workgroup block
                    allc = w.reshape(-1, 4).view(np.int32)
                    if not hits and (allc == v).all(1).any():
                        hits.append("elsewhere in the workgroup")
                    rel[" | ".join(hits) if hits else "no source found"] += 1
    print(f"{len(key)} blocks, {n_bad} wrong float4s")
    for k, v in rel.most_common():
        print(f"  {v:6d}  {k}")
    print("by (side, store u):", sorted(by_u.items()))
    print("by lane quarter:", sorted(by_lane.items()))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/race_dump.npz")
