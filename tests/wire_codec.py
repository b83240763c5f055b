"""numpy restatement of the compressed wire (raymarching_amd/csrc/rm_wire.hip):
the byte-exact message layout the GPU encoder writes, and its decoder.  Test
helper for tests/test_wire.py (the codec is this build's own format; the
reference sends no frames between processes)."""
import numpy as np

SEG_WORDS = 25


def _zigzag(d):
    s = ((d & 255).astype(np.int16) ^ 128) - 128  # int8 wrap
    return np.where(s >= 0, 2 * s, -2 * s - 1).astype(np.uint32)


def _header_bytes(n, S):
    return 8 + ((4 * n + 7) & ~7) + ((n * S + 7) & ~7)


def encode(rows):
    """rows: uint32 [n, W] RGBA8 words -> message bytes (uint8 array)."""
    rows = np.ascontiguousarray(rows, np.uint32)
    n, W = rows.shape
    S = (W + 63) // 64
    pad = np.concatenate([rows, np.repeat(rows[:, -1:], S * 64 - W, axis=1)], axis=1) if S * 64 > W else rows
    seg = pad.reshape(n, S, 64)
    counts = np.zeros((n, S), np.uint8)
    words = []
    row_words = np.zeros(n, np.uint64)
    for j in range(n):
        for k in range(S):
            p = seg[j, k]
            hdr = int(p[0]) & 0xFFFFFF
            planes = []
            bs = []
            for c in range(3):
                ch = ((p >> (8 * c)) & 255).astype(np.int32)
                z = np.zeros(64, np.uint32)
                z[1:] = _zigzag(ch[1:] - ch[:-1])
                b = int(z.max()).bit_length()
                bs.append(b)
                for i in range(b):
                    bits = ((z >> i) & 1).astype(np.uint64)
                    planes.append(int(np.sum(bits << np.arange(64, dtype=np.uint64))))
            hdr |= (bs[0] << 24) | (bs[1] << 28) | (bs[2] << 32)
            counts[j, k] = 1 + len(planes)
            words.append([hdr] + planes)
            row_words[j] += 1 + len(planes)
    row_off = np.concatenate([[0], np.cumsum(row_words)[:-1]]).astype(np.uint32) if n else np.zeros(0, np.uint32)
    hb = _header_bytes(n, S)
    total_words = int(row_words.sum())
    out = np.zeros(hb + 8 * total_words, np.uint8)
    out[:8] = np.frombuffer(np.array([hb + 8 * total_words], np.int64).tobytes(), np.uint8)
    out[8:8 + 4 * n] = np.frombuffer(row_off.tobytes(), np.uint8)
    c0 = 8 + ((4 * n + 7) & ~7)
    out[c0:c0 + n * S] = counts.ravel()
    flat = np.array([w for seg_words in words for w in seg_words], np.uint64)
    out[hb:] = np.frombuffer(flat.tobytes(), np.uint8)
    return out


def decode(msg, n, W):
    """message -> uint32 [n, W] RGBA8 words (alpha 255)."""
    msg = np.asarray(msg, np.uint8)
    S = (W + 63) // 64
    hb = _header_bytes(n, S)
    row_off = np.frombuffer(msg[8:8 + 4 * n].tobytes(), np.uint32)
    c0 = 8 + ((4 * n + 7) & ~7)
    counts = msg[c0:c0 + n * S].reshape(n, S)
    payload = np.frombuffer(msg[hb:].tobytes(), np.uint64)
    out = np.zeros((n, S * 64), np.uint32)
    lanes = np.arange(64, dtype=np.uint64)
    for j in range(n):
        off = int(row_off[j])
        for k in range(S):
            w = payload[off:off + int(counts[j, k])]
            off += int(counts[j, k])
            h = int(w[0])
            bs = [(h >> 24) & 15, (h >> 28) & 15, (h >> 32) & 15]
            q = 1
            px = np.zeros(64, np.uint32)
            for c in range(3):
                z = np.zeros(64, np.uint32)
                for i in range(bs[c]):
                    z |= (((np.uint64(w[q]) >> lanes) & np.uint64(1)).astype(np.uint32)) << np.uint32(i)
                    q += 1
                d = ((z >> 1).astype(np.int64) ^ -(z & 1).astype(np.int64))
                d[0] = (h >> (8 * c)) & 255
                px |= ((np.cumsum(d) & 255).astype(np.uint32)) << np.uint32(8 * c)
            out[j, 64 * k:64 * k + 64] = px | np.uint32(0xFF000000)
    return out[:, :W]
