/*
 * oracle/selftest.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A driver for the CPU restatement built with AddressSanitizer and
 * UndefinedBehaviorSanitizer (oracle/Makefile target `sanitize`,
 * tests/test_oracle_kat.py): renders small frames of every scene, the
 * diagnostic channels, FXAA and bloom over ragged sizes, so out-of-bounds
 * accesses, overflows and other UB in the restatement abort the run.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct {
    float res_x, res_y, mouse_x, mouse_y, pos_x, pos_y, pos_z, time;
    int32_t max_steps, shadow_max_steps;
    float jit_x, jit_y;
} oracle_uniforms;

int oracle_render(int scene, const oracle_uniforms *u, int W, int H, int row0, int nrows, float *out, uint32_t *evals);
int oracle_render_diag(int scene, const oracle_uniforms *u, int W, int H, int row0, int nrows, float *diag, float *out);
int oracle_fxaa(int W, int H, const uint32_t *in, uint32_t *out, float *out_f32);
int oracle_bloom(int W, int H, const uint32_t *in, uint32_t *out, uint32_t *mips);

int main(void) {
    const int sizes[][2] = {{1, 1}, {7, 3}, {33, 17}, {64, 40}};
    const float poses[][6] = {{2, 3, 3, 0, 0, 0}, {2.1476f, 3.0392f, 5.6605f, -0.5881f, 0.1508f, 162.79f},
                              {-4.5641f, 3.4868f, 5.1230f, -0.7137f, -0.1078f, 6.8974f}};
    long checked = 0;
    for (int si = 0; si < 4; si++)
        for (int pi = 0; pi < 3; pi++)
            for (int scene = 0; scene < 4; scene++) {
                const int W = sizes[si][0], H = sizes[si][1];
                const float *p = poses[pi];
                oracle_uniforms u = {(float)W, (float)H, p[3], p[4], p[0], p[1], p[2], p[5], 64, scene == 2 ? 32 : 0, 0.0f, 0.0f};
                float *img = malloc(sizeof(float) * 4 * W * H);
                uint32_t *ev = malloc(sizeof(uint32_t) * W * H);
                if (oracle_render(scene, &u, W, H, 0, H, img, ev)) return 1;
                if (scene >= 2) {
                    float *d = malloc(sizeof(float) * 28 * W * H);
                    if (oracle_render_diag(scene, &u, W, H, 0, H, d, img)) return 1;
                    free(d);
                }
                uint32_t *px = malloc(sizeof(uint32_t) * W * H), *o = malloc(sizeof(uint32_t) * W * H);
                for (int i = 0; i < W * H; i++) {
                    float c = img[4 * i];
                    px[i] = (c == c ? (uint32_t)(fminf(fmaxf(c, 0.0f), 1.0f) * 255.0f) : 0u) * 0x010101u | 0xff000000u;
                }
                if (oracle_fxaa(W, H, px, o, NULL) || oracle_bloom(W, H, px, o, NULL)) return 1;
                checked += W * H;
                free(img), free(ev), free(px), free(o);
            }
    printf("selftest ok: %ld pixels\n", checked);
    return 0;
}
