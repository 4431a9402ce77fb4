"""CPU checks of the LDS image addressing of the C5 gradient pass
(dmdqn_amd/csrc/learn_shared.hip): every call site of hsplit computes exactly
hoff(r, c) for the (row, column) it means, and the images stay bijective.  A
wrong split reads another wave's columns (a race, not a fault), so it is
checked here on every lane / index the kernel uses, not by a spot check."""
import itertools

H, DP = 128, 96


def hoff(r, c, LD=H):
    ch = c >> 3
    return (8 * LD * (r >> 3) + 256 * (ch >> 2) + 32 * (r & 7) +
            8 * ((ch & 3) ^ (((r >> 1) & 1) | ((r >> 2) & 2))) + (c & 7))


def hsplit(rlo, clo, rblk, cblk, LD=H):
    return hoff(rlo, clo, LD) + 16 * LD * rblk + 256 * cblk


def test_hoff_bijective():
    for LD in (H, DP):
        offs = {hoff(r, c, LD) for r in range(128) for c in range(LD)}
        assert len(offs) == 128 * LD and max(offs) < 128 * LD


def test_frag_tr_h_split():
    # frag_tr_h: lane (i, g) first read = row r0 + 8g + (i >> 2), column c0 + 4(i & 3)
    for LD, cmax in ((H, H), (DP, DP)):
        for r0, c0 in itertools.product(range(0, 128, 32), range(0, cmax, 16)):
            for lane in range(64):
                i, g = lane & 15, lane >> 4
                split = hsplit(8 * (g & 1) + (i >> 2), (c0 & 16) + 4 * (i & 3), g >> 1, 0, LD) + \
                    (16 * LD * (r0 >> 4) + 256 * (c0 >> 5))
                r, c = r0 + 8 * g + (i >> 2), c0 + 4 * (i & 3)
                assert split == hoff(r, c, LD)
                # the second read, 4 rows down, is the first + 128 elements
                assert split + 128 == hoff(r + 4, c, LD)


def test_row_write_split():
    for w, lane, t in itertools.product(range(8), range(64), range(8)):
        i, g = lane & 15, lane >> 4
        row = 16 * w + i
        assert hsplit(i, 16 * (t & 1) + 4 * g, w, 0) + 256 * (t >> 1) == hoff(row, 16 * t + 4 * g)
        if t < 3:  # the X image, LD 96, column 32s + 8g
            assert hsplit(i, 8 * g, w, 0, DP) + 256 * t == hoff(row, 32 * t + 8 * g, DP)


def test_dz2_conversion_split():
    for w, lane, j in itertools.product(range(8), range(64), range(4)):
        b, k0 = (lane >> 1) + 32 * j, 16 * w + 8 * (lane & 1)
        split = hsplit((lane >> 1) & 15, 16 * (w & 1) + 8 * (lane & 1), lane >> 5, w >> 1) + 16 * H * 2 * j
        assert split == hoff(b, k0)
