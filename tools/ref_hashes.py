#!/usr/bin/env python3
"""Fingerprints of the reference's shader files, for rm_load_scene's reload
semantics (raymarching_amd/csrc/rm_capi.cpp, "scene files of registered
names").  Build container only (reads /root/reference); prints the constants
rm_capi.cpp holds.  Only 64-bit hashes are kept, never the text.

A fingerprint is FNV-1a 64 over the file's bytes with every whitespace byte
removed (line endings and indentation do not matter).  output_shader.frag is
split in three parts: the prelude up to and including the line that includes
common.frag, the scene part (materials, floorMat, sceneSDF: up to the brace
that closes sceneSDF) and the pipeline part (the rest: hashes, light, render,
main).
"""
import sys

WS = b" \t\r\n\v\f"


def fnv1a64(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for b in data:
        if b in WS:
            continue
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def split_scene(text: bytes):
    """(prelude, scene, pipeline) of an output_shader.frag-shaped file, or None."""
    k = text.find(b"#include")
    if k < 0:
        return None
    e = text.find(b"\n", k)
    e = len(text) if e < 0 else e + 1
    s = text.find(b"sceneSDF(", e)
    s = text.find(b"{", s) if s >= 0 else -1
    if s < 0:
        return None
    depth = 0
    for i in range(s, len(text)):
        c = text[i:i + 1]
        if c == b"{":
            depth += 1
        elif c == b"}":
            depth -= 1
            if depth == 0:
                return text[:e], text[e:i + 1], text[i + 1:]
    return None


def main(ref="/root/reference"):
    o = open(f"{ref}/output_shader.frag", "rb").read()
    pre, scene, pipe = split_scene(o)
    print(f"kRefCommon   = 0x{fnv1a64(open(f'{ref}/common.frag', 'rb').read()):016x}ULL")
    print(f"kRefTemplate = 0x{fnv1a64(open(f'{ref}/template.frag', 'rb').read()):016x}ULL")
    print(f"kRefOScene   = 0x{fnv1a64(scene):016x}ULL")
    print(f"kRefOFrame   = 0x{fnv1a64(pre + pipe):016x}ULL  (prelude + pipeline)")


if __name__ == "__main__":
    main(*sys.argv[1:])
