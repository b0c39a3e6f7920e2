/* sanitize_check.c — AddressSanitizer / UBSan driver for the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Builds seeded ragged batches in exactly-sized heap buffers (so any out-of-bounds index in walker_oracle.c hits
 * a redzone) and steps them through every mode the oracle has: the engine spring and the G2 / G3 elements, string
 * springs, pinned masses, run1 / run2, continuous and discrete actions, G1 friction, and the gravity / coulomb /
 * bounce pair passes; then observe and reset.  Build and run: `make -C oracle sanitize` (tests/test_oracle_sanitize.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "walker_oracle.h"

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t)(rs >> 11); }
static float unif(float a, float b) { return a + (b - a) * (float)(rnd() % 1000000) / 1000000.f; }
static void *xmalloc(size_t n) { void *p = malloc(n ? n : 1); if (!p) { perror("malloc"); exit(2); } return p; }

static int run_case(int N, int spring_mode, int pair_mode, int integrator, int action_mode, int friction_mode,
                    int in3d, int conmid, int subset) {
    int32_t *mass_off = xmalloc(sizeof(int32_t) * (N + 1)), *edge_off = xmalloc(sizeof(int32_t) * (N + 1));
    int32_t *muscle_off = xmalloc(sizeof(int32_t) * (N + 1));
    mass_off[0] = edge_off[0] = muscle_off[0] = 0;
    for (int w = 0; w < N; w++) {
        const int M = 1 + (int)(rnd() % 20), K = M > 1 ? (int)(rnd() % (2 * M)) : 0, A = K / 3;
        mass_off[w + 1] = mass_off[w] + M;
        edge_off[w + 1] = edge_off[w] + K;
        muscle_off[w + 1] = muscle_off[w] + A;
    }
    const int P = mass_off[N], E = edge_off[N], U = muscle_off[N];
    float *pos = xmalloc(sizeof(float) * 3 * P), *vel = xmalloc(sizeof(float) * 3 * P), *acc = xmalloc(sizeof(float) * 3 * P);
    float *m = xmalloc(sizeof(float) * P);
    uint8_t *contact = xmalloc(P), *pinned = xmalloc(P);
    double *charge = xmalloc(sizeof(double) * P), *radius = xmalloc(sizeof(double) * P);
    uint8_t *bounce_set = subset ? xmalloc(P) : NULL;   /* Point.bounce(k, other=<list>): caller / list bits */
    for (int i = 0; i < P; i++) {
        if (bounce_set) bounce_set[i] = (uint8_t)(rnd() & 3);
        for (int c = 0; c < 3; c++) { pos[3 * i + c] = unif(-20.f, 20.f); vel[3 * i + c] = unif(-1.f, 1.f); acc[3 * i + c] = 0.f; }
        if (!in3d) { pos[3 * i + 2] = 0.f; vel[3 * i + 2] = 0.f; }
        m[i] = unif(0.5f, 5.f);
        pinned[i] = (rnd() % 17) == 0;
        charge[i] = unif(-3.f, 3.f);
        radius[i] = pow((double)m[i], 0.3);
    }
    int32_t *ei = xmalloc(sizeof(int32_t) * E), *ej = xmalloc(sizeof(int32_t) * E);
    float *rest = xmalloc(sizeof(float) * E), *k = xmalloc(sizeof(float) * E), *c = xmalloc(sizeof(float) * E);
    uint8_t *flags = xmalloc(E);
    for (int w = 0; w < N; w++) {
        const int M = mass_off[w + 1] - mass_off[w];
        for (int e = edge_off[w]; e < edge_off[w + 1]; e++) {
            ei[e] = (int)(rnd() % M);
            ej[e] = (ei[e] + 1 + (int)(rnd() % (M - 1))) % M;
            rest[e] = unif(1.f, 15.f); k[e] = unif(100.f, 2000.f); c[e] = unif(0.f, 20.f);
            flags[e] = (rnd() % 5) == 0;
        }
    }
    float *mx = xmalloc(sizeof(float) * U), *minl = xmalloc(sizeof(float) * U), *maxl = xmalloc(sizeof(float) * U);
    float *stride = xmalloc(sizeof(float) * U);
    for (int w = 0; w < N; w++)
        for (int u = muscle_off[w], e = edge_off[w]; u < muscle_off[w + 1]; u++, e++) {
            mx[u] = rest[e]; minl[u] = 0.1f * rest[e]; maxl[u] = 1.5f * rest[e]; stride[u] = 2.f;
        }
    int32_t *steps = xmalloc(sizeof(int32_t) * N);
    memset(steps, 0, sizeof(int32_t) * N);
    int Amax = 0, Dmax = 0;
    for (int w = 0; w < N; w++) {
        const int A = muscle_off[w + 1] - muscle_off[w], M = mass_off[w + 1] - mass_off[w];
        if (A > Amax) Amax = A;
        const int D = 3 * (in3d ? 3 : 2) * M + (conmid ? 3 : 0) + A;
        if (D > Dmax) Dmax = D;
    }
    const int cols = Amax > 0 ? Amax : 1;
    float *action = xmalloc(sizeof(float) * N * cols);
    float *obs = xmalloc(sizeof(float) * N * Dmax), *reward = xmalloc(sizeof(float) * N);
    uint8_t *done = xmalloc(N);
    float *centroid = xmalloc(sizeof(float) * 3 * N), *energy = xmalloc(sizeof(float) * N);
    float *noise = xmalloc(sizeof(float) * 3 * P);
    for (int i = 0; i < 3 * P; i++) noise[i] = unif(-0.1f, 0.1f);

    orc_params p;
    memset(&p, 0, sizeof p);
    p.g = 100; p.ground = 0; p.groundk = 1000; p.grounddamp = 100; p.friction = 100; p.dt = 0.01;
    p.pk = p.vk = p.ak = p.mk = 1; p.in3d = in3d; p.max_steps = 1000; p.midform = 1; p.conmid = conmid;
    p.spring_mode = spring_mode; p.action_mode = action_mode; p.integrator = integrator; p.pair_mode = pair_mode;
    p.pair_g = 9.8; p.pair_k = 1e4; p.pair_e = 16e-20; p.bounce_k = 100;
    p.g3_gravity[1] = -9.8; p.g3_damping = 0.99; p.g3_air = 0.01; p.g3_ground_level = -50; p.g3_restitution = 0.8;
    p.g3_friction = 0.5; p.g3_ground = 1; p.friction_mode = friction_mode;
    orc_batch b = {N, mass_off, edge_off, muscle_off, pos, vel, acc, m, ei, ej, rest, k, c, flags, mx, minl, maxl,
                   stride, steps, contact, pinned, charge, radius, bounce_set};
    orc_out o = {obs, Dmax, reward, done, centroid, energy};
    int rc = orc_reset(&b, &p, noise, 1);
    for (int s = 0; s < 8 && rc == 0; s++) {
        for (int i = 0; i < N * cols; i++) action[i] = action_mode ? (float)(rnd() & 1) : unif(-1.f, 1.f);
        rc = orc_step(&b, &p, action, Amax, cols, &o, 1);
    }
    if (rc == 0) rc = orc_observe(&b, &p, &o, 1);
    int finite = 0;
    for (int i = 0; i < N; i++) finite += isfinite(reward[i]) != 0;
    printf("case spring=%d pair=%d%s run%d act=%d fric=%d in3d=%d conmid=%d: rc=%d, %d/%d finite rewards\n",
           spring_mode, pair_mode, subset ? " (bounce subset)" : "", integrator == 2 ? 2 : 1, action_mode, friction_mode,
           in3d, conmid, rc, finite, N);
    free(mass_off); free(edge_off); free(muscle_off); free(pos); free(vel); free(acc); free(m); free(contact);
    free(pinned); free(charge); free(radius); free(bounce_set); free(ei); free(ej); free(rest); free(k); free(c); free(flags); free(mx);
    free(minl); free(maxl); free(stride); free(steps); free(action); free(obs); free(reward); free(done);
    free(centroid); free(energy); free(noise);
    return rc;
}

int main(void) {
    int bad = 0;
    bad |= run_case(60, 0, 0, 1, 0, 0, 1, 0, 0) != 0;
    bad |= run_case(60, 0, 7, 1, 0, 0, 1, 1, 0) != 0;
    bad |= run_case(60, 0, 4, 1, 0, 0, 1, 0, 1) != 0;
    bad |= run_case(60, 1, 0, 2, 1, 0, 0, 0, 0) != 0;
    bad |= run_case(60, 2, 0, 1, 0, 0, 1, 0, 0) != 0;
    bad |= run_case(60, 0, 3, 2, 0, 1, 0, 1, 0) != 0;
    printf(bad ? "FAILED\n" : "sanitize ok\n");
    return bad;
}
