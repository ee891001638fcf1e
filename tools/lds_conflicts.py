"""LDS bank-conflict model of conv3h's fragment reads (va_seg.hip conv3h_kernel), per ds_read_b128 lane group.

ds_read_b128 serves a wave in four 16-lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32;
MI355X_MICROARCH.md §LDS); a group is conflict-free when its 16 addresses fall in 16 distinct 16-byte slots of the
256-byte bank row.  Rows are 96 bytes (16 channels x 3 bf16 planes).  Checked:
  A (weights): row r = channel, chunk c in slot c ^ ((r >> 3) & 1)
  B (halo):    B-block row r -> pixel t3h_perm(r) of the TH x TW tile; tap (ky, kx) reads halo pixel
               (py + ky, px + kx), chunk c in slot c ^ ((hy ^ ((hx >> 3) & (TW >= 16))) & 1)
for TW = 4, 8, 16, 32 and 3x3 / 2x2 taps.  Prints the worst and mean conflict degree (1 = conflict-free).
usage: python tools/lds_conflicts.py"""
from collections import defaultdict

G = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)), list(range(4, 12)) + list(range(16, 20)) +
     list(range(28, 32))]
G = G + [[x + 32 for x in g] for g in G]
ROW = 96


def perm(r):
    return r if r < 4 else r + 12 if r < 12 else r - 8 if r < 16 else r + 8 if r < 20 else r - 12 if r < 28 else r


def degree(addrs):
    out = []
    for g in G:
        d = defaultdict(set)
        for lane in g:
            d[(addrs[lane] // 16) % 16].add(addrs[lane])
        out.append(max(len(v) for v in d.values()))
    return out


def a_reads():
    degs = []
    for base in (0, 32, 64, 96):
        for p in range(3):
            addrs = [(base + (l & 31)) * ROW + 16 * ((3 * (l >> 5) + p) ^ (((base + (l & 31)) >> 3) & 1))
                     for l in range(64)]
            degs += degree(addrs)
    return degs


def b_reads(tw, kh, kw):
    hw, xm = tw + kw - 1, 1 if tw >= 16 else 0
    degs = []
    for wm in range(2):
        for jb in range(2):
            for ky in range(kh):
                for kx in range(kw):
                    for p in range(3):
                        addrs = []
                        for l in range(64):
                            q = wm * 64 + 32 * jb + perm(l & 31)
                            hy, hx = q // tw + ky, q % tw + kx
                            addrs.append((hy * hw + hx) * ROW + 16 * ((3 * (l >> 5) + p) ^ ((hy ^ ((hx >> 3) & xm)) & 1)))
                        degs += degree(addrs)
    return degs


def main():
    d = a_reads()
    print(f"A reads: worst {max(d)}, mean {sum(d) / len(d):.3f}")
    for tw in (4, 8, 16, 32):
        for kh, kw in ((3, 3), (2, 2)):
            d = b_reads(tw, kh, kw)
            print(f"B halo reads TW={tw:2d} {kh}x{kw}: worst {max(d)}, mean {sum(d) / len(d):.3f}")


if __name__ == "__main__":
    main()
