"""numpy restatement of the compressed wire (raymarching_amd/csrc/rm_wire_tile.h,
rm_wire.hip): the byte-exact message layout the GPU encoders write (rows
encoder and render epilogue), and its decoder.  Test helper for
tests/test_wire.py (the codec is this build's own format; the reference sends
no frames between processes).

A part of n packed RGBA8 rows of W pixels in 8x8 tiles (TX = ceil(W/8) across,
TY = ceil(n/8) down, tile t = ty TX + tx; pixels outside the part are the word
0).  Per tile and channel: differences to the left neighbour, to the one above
in the first column, mod 256 as int8, zig-zagged; the width b of the largest;
the header word (lane 0's RGB, b_R << 24, b_G << 28, b_B << 32) and b bit planes
per channel (bit l = lane (l & 7, l >> 3)).  Message: int64 bytes, uint32 per
tile (word offset << 5 | word count), padded to 8 B, then the tiles' words in
order."""
import numpy as np

TILE_WORDS = 25


def _zigzag(d):
    s = ((d & 255).astype(np.int16) ^ 128) - 128  # int8 wrap
    return np.where(s >= 0, 2 * s, -2 * s - 1).astype(np.uint32)


def header_bytes(T):
    return 8 + ((4 * T + 7) & ~7)


def _tiles(rows):
    n, W = rows.shape
    TX, TY = (W + 7) // 8, (n + 7) // 8
    pad = np.zeros((TY * 8, TX * 8), np.uint32)
    pad[:n, :W] = rows
    return pad.reshape(TY, 8, TX, 8).transpose(0, 2, 1, 3).reshape(TY * TX, 64), TX, TY


def tile_words(p):
    """The words of one tile: p = uint32 [64] RGBA8, lane l = (col l & 7, row l >> 3)."""
    planes, bs = [], []
    for c in range(3):
        v = ((p >> (8 * c)) & 255).astype(np.int32).reshape(8, 8)
        ref = np.empty_like(v)
        ref[:, 1:] = v[:, :-1]
        ref[1:, 0] = v[:-1, 0]
        ref[0, 0] = v[0, 0]
        z = _zigzag((v - ref).ravel())
        z[0] = 0
        b = int(z.max()).bit_length()
        bs.append(b)
        for i in range(b):
            bits = ((z >> i) & 1).astype(np.uint64)
            planes.append(int(np.sum(bits << np.arange(64, dtype=np.uint64))))
    hdr = (int(p[0]) & 0xFFFFFF) | (bs[0] << 24) | (bs[1] << 28) | (bs[2] << 32)
    return [hdr] + planes


def encode(rows):
    """rows: uint32 [n, W] RGBA8 words -> message bytes (uint8 array)."""
    rows = np.ascontiguousarray(rows, np.uint32)
    tiles, TX, TY = _tiles(rows)
    T = TX * TY
    words = [tile_words(tiles[t]) for t in range(T)]
    counts = np.array([len(w) for w in words], np.int64)
    offs = (np.concatenate([[0], np.cumsum(counts)[:-1]]) if T else np.zeros(0)).astype(np.int64)
    table = ((offs << 5) | counts).astype(np.uint32)
    hb = header_bytes(T)
    total = int(counts.sum())
    out = np.zeros(hb + 8 * total, np.uint8)
    out[:8] = np.frombuffer(np.array([hb + 8 * total], np.int64).tobytes(), np.uint8)
    out[8:8 + 4 * T] = np.frombuffer(table.tobytes(), np.uint8)
    flat = np.array([x for w in words for x in w], np.uint64)
    out[hb:] = np.frombuffer(flat.tobytes(), np.uint8)
    return out


def decode(msg, n, W):
    """message -> uint32 [n, W] RGBA8 words (alpha 255)."""
    msg = np.asarray(msg, np.uint8)
    TX, TY = (W + 7) // 8, (n + 7) // 8
    T = TX * TY
    hb = header_bytes(T)
    offs = np.frombuffer(msg[8:8 + 4 * T].tobytes(), np.uint32) >> 5
    payload = np.frombuffer(msg[hb:].tobytes(), np.uint64)
    out = np.zeros((TY * 8, TX * 8), np.uint32)
    lanes = np.arange(64, dtype=np.uint64)
    for t in range(T):
        w = payload[int(offs[t]):]
        h = int(w[0])
        bs = [(h >> 24) & 15, (h >> 28) & 15, (h >> 32) & 15]
        q = 1
        px = np.zeros(64, np.uint32)
        for c in range(3):
            z = np.zeros(64, np.uint32)
            for i in range(bs[c]):
                z |= (((np.uint64(w[q]) >> lanes) & np.uint64(1)).astype(np.uint32)) << np.uint32(i)
                q += 1
            d = ((z >> 1).astype(np.int64) ^ -(z & 1).astype(np.int64)).reshape(8, 8)
            d[0, 0] = (h >> (8 * c)) & 255
            v = np.cumsum(d, axis=1) + (np.cumsum(d[:, 0]) - d[:, 0])[:, None]
            px |= ((v.ravel() & 255).astype(np.uint32)) << np.uint32(8 * c)
        ty, tx = divmod(t, TX)
        out[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8] = (px | np.uint32(0xFF000000)).reshape(8, 8)
    return out[:n, :W]
