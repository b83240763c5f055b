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
