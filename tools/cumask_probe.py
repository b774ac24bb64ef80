import ctypes, os, collections
rs = ctypes.CDLL(os.path.join("tools", "probe", "librccl_shape.so"))
def where(bits, blocks=64, ncu=256):
    words = (ctypes.c_uint * 8)()
    for b in bits: words[b // 32] |= 1 << (b % 32)
    out = (ctypes.c_uint * (2 * blocks))()
    assert rs.rs_where(words, 8, blocks, out) == 0
    locs = collections.Counter()
    for q in range(blocks):
        x, h = out[2*q], out[2*q+1]
        locs[(x & 0xf, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 0xf)] += 1
    return sorted(locs)
for bits in ([0], [1], [2], [7], [8], [9], [31], [32], [63], [64], [128], [255], list(range(0, 8)), list(range(248, 256)), list(range(0,256,32))):
    print(bits if len(bits) < 3 else "%d..%d step %d" % (bits[0], bits[-1], bits[1]-bits[0]), "->", where(bits))
