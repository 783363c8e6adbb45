"""Exhaustive bank check of the B16 LDS image (gemm_split.hip b16_off): for every 32-row
fragment block of a 256-row image and every chunk q = 2 p + h, the 16-lane groups of a
ds_read_b128 (MI355X_MICROARCH.md, LDS table) must hit 16 distinct 16-B slots of the 256-B
bank row; and the swizzle must be an involution inside each 256-B block (so each 1-KiB DMA
instruction reads exactly one contiguous KiB of source).  Pure CPU."""


def sw(blk):
    m = blk % 6
    return 14 if m in (0, 4, 5) else 13


def off_chunk(r, q):
    c = 6 * r + q
    return c ^ sw(c >> 4)


def main():
    groups = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32))]
    for r0 in range(0, 256, 32):
        for q in range(6):
            for G in groups:
                slots = {off_chunk(r0 + l, q) % 16 for l in G}
                assert len(slots) == 16, (r0, q, G)
    for c in range(6 * 256):
        x = c ^ sw(c >> 4)
        assert x >> 4 == c >> 4 and x ^ sw(x >> 4) == c
    print('B16 swizzle: conflict-free fragment reads, involution within 256-B blocks: OK')


if __name__ == '__main__':
    main()
