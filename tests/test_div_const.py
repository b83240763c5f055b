"""The scene library divides by constants with one Markstein correction of
x * RN(1/k) (rm_device.h div_const; rm_sdf_lib.h div_k) and relies on it being
the correctly rounded quotient.  Checked here exhaustively over two binades of x
(every mantissa, both relative positions of the mantissas) for the divisors the
library and the scenes use, on the host with the same float operations."""
import os
import subprocess
import tempfile

import pytest

SRC = r'''
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static float div_const(float x, float b, float rb) { float q = x * rb; float r = fmaf(-b, q, x); return fmaf(r, rb, q); }
int main(void) {
    const float bs[] = {3.0f, 9.0f, 27.0f, 0.33f, 0.5f, 0.25f, 0.1f, 0.7f, 1.3f};
    long bad = 0;
    for (unsigned k = 0; k < sizeof(bs) / sizeof(bs[0]); k++) {
        const float b = bs[k], rb = 1.0f / b;
        for (uint32_t e = 0; e < 2; e++)
            for (uint32_t m = 0; m < (1u << 23); m++) {
                uint32_t u = ((127u + e) << 23) | m;
                float x, got;
                memcpy(&x, &u, 4);
                volatile float ref = x / b;
                got = div_const(x, b, rb);
                if (memcmp(&got, (const void *)&ref, 4)) bad++;
            }
    }
    printf("%ld\n", bad);
    return 0;
}
'''


def test_div_const_is_correctly_rounded():
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "t.c"), os.path.join(d, "t")
        open(c, "w").write(SRC)
        try:
            subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, c, "-lm"], check=True, capture_output=True)
        except (OSError, subprocess.CalledProcessError) as e:
            pytest.skip(f"no host C compiler: {e}")
        out = subprocess.run([exe], check=True, capture_output=True, text=True, timeout=120).stdout
        assert int(out.strip()) == 0


# rm_device.h div_magic / div_by: the launch's row and tile divisions as one
# 32-bit high multiply.  Compiled from the header's own host-callable
# div_magic (a HIP header: hipcc host compile), checked against integer
# division for every divisor up to 4096 at its largest allowed dividend range
# (the bound div_magic accepts), on the range's last 2^16 dividends and a
# stride through the rest.
MAGIC_SRC = r'''
#include <stdint.h>
#include <stdio.h>
#include "rm_device.h"
int main(void) {
    long bad = 0, checked = 0, used = 0;
    for (uint32_t d = 1; d <= 4096; d++) {
        // the largest a_end div_magic accepts for d
        uint64_t lo = 1, hi = (1ull << 32);
        while (lo < hi) { uint64_t mid = (lo + hi + 1) / 2; if (rm::div_magic(d, mid)) lo = mid; else hi = mid - 1; }
        const uint32_t m = rm::div_magic(d, lo);
        if (!m) { if (d >= 2) bad++; continue; }
        used++;
        for (uint64_t a = 0; a < lo; a += (a + 65536 < lo ? 977 : 1)) {
            const uint32_t q = (uint32_t)(((uint64_t)a * m) >> 32);
            checked++;
            if (q != (uint32_t)(a / d)) bad++;
        }
    }
    printf("%ld %ld %ld\n", bad, checked, used);
    return 0;
}
'''


def test_div_magic_is_floor_division():
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raymarching_amd", "csrc")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "m.cpp"), os.path.join(d, "m")
        open(src, "w").write(MAGIC_SRC)
        subprocess.run([hipcc, "-O2", "-x", "hip", "--offload-arch=gfx950", "-I", inc, src, "-o", exe], check=True,
                       capture_output=True, timeout=300)
        bad, checked, used = map(int, subprocess.run([exe], check=True, capture_output=True, text=True,
                                                     timeout=600).stdout.split())
    assert used == 4095 and checked > 10_000_000 and bad == 0, (bad, checked, used)
