/* walker_oracle.c — plain-C restatement of the reference CPU walker step.
 *
 *   TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 *   may load this library, and only as the checker / the reported CPU baseline.  The product path
 *   (walker_gym_amd + libwalker_hip.so) never links or calls it.
 *
 * Parity pin: the tests/golden fixtures, produced by running the reference's own code
 * (tests/golden/make_golden.py).  This restatement reproduces numpy 2.2's mixed-precision
 * arithmetic op by op, so it matches those goldens bit for bit (tests/test_oracle_golden.py).
 *
 * numpy semantics being restated (NEP 50, numpy >= 2):
 *   - float32 array (op) Python scalar  -> float32 op, the scalar rounded to float32 first;
 *   - np.linalg.norm(float32[3])        -> OpenBLAS sdot: float32 products summed in double,
 *                                           rounded to float32, then float32 sqrt;
 *   - gym/engine.py:73 `.astype(float)` makes the distance a float64 scalar, so the spring force
 *     `-f_size * direction / distance` (engine.py:75) and `f / self.m` (engine.py:67) are float64;
 *     `a += f64` adds in double and rounds to float32 (same_kind in-place cast);
 *   - np.mean / np.sum of a float32 list -> numpy pairwise summation in float32.
 * Compiled with -O2 -ffp-contract=off (no FMA contraction, SSE float arithmetic).
 */
#include "walker_oracle.h"

#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_ABI 5
int orc_abi_version(void) { return ORC_ABI; }

/* Config.r (gym/engine.py:9, gym/optimized_engine.py:7): the distance clamp, a Python float. */
static const double CONFIG_R = 16e-36;

/* np.linalg.norm(v) for a float32 3-vector (gym/engine.py:73,86; gym/optimized_walker.py:25). */
static float np_norm3(float x, float y, float z) {
    float px = x * x, py = y * y, pz = z * z;
    double s = 0.0;
    s += (double)px; s += (double)py; s += (double)pz;
    return sqrtf((float)s);
}
float orc_np_norm3(const float *v) { return np_norm3(v[0], v[1], v[2]); }

/* np.dot(float32[3], float32[3]) (gym/optimized_walker.py:64,103): same sdot kernel. */
static float np_dot3(float ax, float ay, float az, float bx, float by, float bz) {
    float p0 = ax * bx, p1 = ay * by, p2 = az * bz;
    double s = 0.0;
    s += (double)p0; s += (double)p1; s += (double)p2;
    return (float)s;
}

/* numpy's float32 pairwise summation (add.reduce inner loop), used by np.mean/np.sum. */
static float pairwise(const float *a, int64_t n, int64_t st) {
    if (n < 8) {
        float res = 0.f;
        for (int64_t i = 0; i < n; i++) res += a[i * st];
        return res;
    } else if (n <= 128) {
        float r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j * st];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[(i + j) * st];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i * st];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise(a, n2, st) + pairwise(a + n2 * st, n - n2, st);
    }
}
float orc_np_pairwise_sum(const float *a, int64_t n, int64_t stride) { return pairwise(a, n, stride); }

/* Point.forced with a float64 force (gym/engine.py:65-67 reached from anti_forced :69-76):
 * a(f32) += f(f64) / m  -> computed in double, rounded to float32. */
static inline float add_f64(float a, double f, double m) { return (float)((double)a + f / m); }
/* Point.forced with a float32 force: a += f / m, all float32 (m cast to float32). */
static inline float add_f32(float a, float f, float m) { return a + f / m; }

/* Python builtin max(x, lo) then min(x, hi) as in Muscle.regulation (gym/optimized_walker.py:27-30). */
static inline float regulate(float x, float lo, float hi) {
    if (lo > x) x = lo;
    if (hi < x) x = hi;
    return x;
}

/* spring_mode 2: one G3 Environment.update_physics for walker w (gym/optimized_walker/env.py:135-184), the
 * walker's springs standing for Environment.springs (muscles first, at their Muscle.x rest).  Everything is
 * float32: core.py's anti_forced takes the distance as float32 (:88), so no float64 enters. */
static void walker_step_g3(const orc_batch *b, const orc_params *p, int w) {
    const int m0 = b->mass_off[w], m1 = b->mass_off[w + 1];
    const int e0 = b->edge_off[w], e1 = b->edge_off[w + 1];
    const int u0 = b->muscle_off[w], A = b->muscle_off[w + 1] - u0;
    float *pos = b->pos, *vel = b->vel, *acc = b->acc;
    const float gv[3] = {(float)p->g3_gravity[0], (float)p->g3_gravity[1], (float)p->g3_gravity[2]};
    /* zero (:141-142), then gravity point.forced(self.gravity * point.m) on the env's points (:145-146);
     * DingPoint.zero / forced are no-ops (core.py:269-275): its a stays zeros */
    for (int q = m0; q < m1; q++) {
        const float mf = b->m[q];
        const int pin = b->pinned && b->pinned[q];
        for (int c = 0; c < 3; c++) acc[3 * q + c] = pin ? 0.f : 0.f + (gv[c] * mf) / mf;
    }
    /* springs in list order (:149-150): core.py resilience (:93-122) -> anti_forced (:85-91):
     * current = norm(self - other) (float32); f_size = -(current - x) * k (0 for a slack string);
     * distance = max(norm(direction).astype(float32), Config.r); force = -f_size * direction / distance;
     * forced: a += force / m, all float32 */
    for (int e = e0; e < e1; e++) {
        const int i = m0 + b->ei[e], j = m0 + b->ej[e];
        const float x = (e - e0 < A) ? b->mx[u0 + (e - e0)] : b->rest[e];
        const float *pi = pos + 3 * i, *pj = pos + 3 * j;
        const float cur = np_norm3(pi[0] - pj[0], pi[1] - pj[1], pi[2] - pj[2]);
        const float dx = cur - x;
        const int string = b->flags ? (b->flags[e] & 1) : 0;
        const float fsz = (dx < 0.f && string) ? 0.f : (-dx) * b->k[e];
        const float nf = -fsz;
        const float dist = (CONFIG_R > (double)cur) ? (float)CONFIG_R : cur;
        if (!(b->pinned && b->pinned[i]))
            for (int c = 0; c < 3; c++) acc[3 * i + c] = acc[3 * i + c] + ((nf * (pj[c] - pi[c])) / dist) / b->m[i];
        if (!(b->pinned && b->pinned[j]))
            for (int c = 0; c < 3; c++) acc[3 * j + c] = acc[3 * j + c] + ((nf * (pi[c] - pj[c])) / dist) / b->m[j];
    }
    const float damp = (float)p->g3_damping, dragc = (float)(-0.5 * p->g3_air), dt = (float)p->dt;
    const float level = (float)p->g3_ground_level, rest = (float)p->g3_restitution, fr = (float)p->g3_friction;
    for (int q = m0; q < m1; q++) {
        float *a = acc + 3 * q, *v = vel + 3 * q, *x = pos + 3 * q;
        const float mf = b->m[q];
        const int pin = b->pinned && b->pinned[q];
        if (!pin) {
            /* damping v *= damping (:153-154), then air drag (:157-161): speed = norm(v) (float32);
             * drag = ((-0.5 * air) * speed) * v, the Python float weakly cast to float32 */
            for (int c = 0; c < 3; c++) v[c] = v[c] * damp;
            const float coef = dragc * np_norm3(v[0], v[1], v[2]);
            for (int c = 0; c < 3; c++) a[c] = a[c] + (coef * v[c]) / mf;
        }
        /* Point.run1 over the registry, DingPoints included (core.py:185-200): v += a*t; pos += v*t */
        for (int c = 0; c < 3; c++) v[c] = v[c] + a[c] * dt;
        for (int c = 0; c < 3; c++) x[c] = x[c] + v[c] * dt;
        /* ground (:164-178), env points only: clamp, then bounce with restitution and friction */
        int hit = 0;
        if (!pin && p->g3_ground && x[1] <= level) {
            hit = 1;
            x[1] = level;
            if (v[1] < 0.f) {
                v[1] = (-v[1]) * rest;
                v[0] = v[0] * fr;
                v[2] = v[2] * fr;
            }
        }
        if (b->contact) b->contact[q] = (uint8_t)hit;
    }
    b->steps[w] += 1;
}

static void walker_step(const orc_batch *b, const orc_params *p, int w, const float *action,
                        int32_t action_cols, int32_t action_stride) {
    const int m0 = b->mass_off[w], m1 = b->mass_off[w + 1];
    const int e0 = b->edge_off[w], e1 = b->edge_off[w + 1];
    const int u0 = b->muscle_off[w], A = b->muscle_off[w + 1] - u0;
    float *pos = b->pos, *vel = b->vel, *acc = b->acc;

    /* 1. Creature.act / actdisp (gym/optimized_walker.py:164-172 -> Muscle.act :32-35,
     *    actdisp :37-43, regulation :27-30): only the first min(A, len(a)) muscles act. */
    if (action) {
        int na = A < action_cols ? A : action_cols;
        for (int u = 0; u < na; u++) {
            float x = b->mx[u0 + u];
            float a = action[(int64_t)w * action_stride + u];
            float x0 = b->rest[e0 + u];                       /* originx */
            if (p->action_mode == 1) x = (a != 0.f) ? x + b->stride[u0 + u] : x - b->stride[u0 + u];
            else x = x + a;
            x = regulate(x, x0 * b->minl[u0 + u], x0 * b->maxl[u0 + u]);
            b->mx[u0 + u] = x;
        }
    }

    if (p->spring_mode == 2) {            /* the G3 engine instead of steps 2-5 */
        walker_step_g3(b, p, w);
        return;
    }

    /* 2. zero accelerations (Creature.run, gym/optimized_walker.py:120-121). */
    for (int q = m0; q < m1; q++) acc[3 * q] = acc[3 * q + 1] = acc[3 * q + 2] = 0.f;

    /* 3. spring pass in edge-list order: muscles, then skeletons (gym/optimized_walker.py:124-127). */
    for (int e = e0; e < e1; e++) {
        const int i = m0 + b->ei[e], j = m0 + b->ej[e];
        const float x = (e - e0 < A) ? b->mx[u0 + (e - e0)] : b->rest[e];
        const float k = b->k[e], c = b->c[e];
        const float *pi = pos + 3 * i, *pj = pos + 3 * j, *vi = vel + 3 * i, *vj = vel + 3 * j;
        float *ai = acc + 3 * i, *aj = acc + 3 * j;
        const double mi = b->m[i], mj = b->m[j];
        const float mif = b->m[i], mjf = b->m[j];
        /* current = norm(self.pos - other.pos) (engine.py:86 / optimized_walker.py:48,87) */
        const float cur = np_norm3(pi[0] - pj[0], pi[1] - pj[1], pi[2] - pj[2]);
        const float dx = cur - x;                               /* engine.py:96 */
        if (p->spring_mode == 1) {
            /* G2 element as written (gym/optimized_walker.py:45-67): inverted-sign spring. */
            float fs = (-dx) * k;                               /* :50 */
            float d0 = pj[0] - pi[0], d1 = pj[1] - pi[1], d2 = pj[2] - pi[2];   /* :53 */
            if (cur > 0.f) { d0 = d0 / cur; d1 = d1 / cur; d2 = d2 / cur; }       /* :54-55 */
            float f0 = fs * d0, f1 = fs * d1, f2 = fs * d2;     /* :58 */
            ai[0] = add_f32(ai[0], f0, mif); ai[1] = add_f32(ai[1], f1, mif); ai[2] = add_f32(ai[2], f2, mif);
            aj[0] = add_f32(aj[0], -f0, mjf); aj[1] = add_f32(aj[1], -f1, mjf); aj[2] = add_f32(aj[2], -f2, mjf);
            float dk = np_dot3(vi[0] - vj[0], vi[1] - vj[1], vi[2] - vj[2], d0, d1, d2);  /* :63-64 */
            float dkc = dk * c;
            float g0 = dkc * d0, g1 = dkc * d1, g2 = dkc * d2;  /* :65 */
            ai[0] = add_f32(ai[0], -g0, mif); ai[1] = add_f32(ai[1], -g1, mif); ai[2] = add_f32(ai[2], -g2, mif);
            aj[0] = add_f32(aj[0], g0, mjf); aj[1] = add_f32(aj[1], g1, mjf); aj[2] = add_f32(aj[2], g2, mjf);
            continue;
        }
        /* engine.py resilience (:78-102): f_size = -dx*k, zero for a slack string (:97-100). */
        const int string = b->flags ? (b->flags[e] & 1) : 0;
        float fsz = (dx < 0.f && string) ? 0.f : (-dx) * k;
        const float nf = -fsz;                                   /* -f_size, engine.py:75 */
        double dist = (double)cur;                               /* .astype(float), engine.py:73 */
        if (CONFIG_R > dist) dist = CONFIG_R;                    /* Python max(distance, r), :74 */
        /* self.anti_forced(f_size, other): direction = other.pos - self.pos */
        {
            float f0 = nf * (pj[0] - pi[0]), f1 = nf * (pj[1] - pi[1]), f2 = nf * (pj[2] - pi[2]);
            ai[0] = add_f64(ai[0], (double)f0 / dist, mi);
            ai[1] = add_f64(ai[1], (double)f1 / dist, mi);
            ai[2] = add_f64(ai[2], (double)f2 / dist, mi);
        }
        /* other.anti_forced(f_size, self): direction = self.pos - other.pos */
        {
            float f0 = nf * (pi[0] - pj[0]), f1 = nf * (pi[1] - pj[1]), f2 = nf * (pi[2] - pj[2]);
            aj[0] = add_f64(aj[0], (double)f0 / dist, mj);
            aj[1] = add_f64(aj[1], (double)f1 / dist, mj);
            aj[2] = add_f64(aj[2], (double)f2 / dist, mj);
        }
        /* relative-velocity damping, gym/optimized_walker.py:92-94,102-106 (same code in Muscle.run
         * :53-55,63-67); the golden runs it through Skeleton.run with k = 0. */
        {
            float d0 = pj[0] - pi[0], d1 = pj[1] - pi[1], d2 = pj[2] - pi[2];
            if (cur > 0.f) { d0 = d0 / cur; d1 = d1 / cur; d2 = d2 / cur; }
            float dk = np_dot3(vi[0] - vj[0], vi[1] - vj[1], vi[2] - vj[2], d0, d1, d2);
            float dkc = dk * c;
            float g0 = dkc * d0, g1 = dkc * d1, g2 = dkc * d2;
            ai[0] = add_f32(ai[0], -g0, mif); ai[1] = add_f32(ai[1], -g1, mif); ai[2] = add_f32(ai[2], -g2, mif);
            aj[0] = add_f32(aj[0], g0, mjf); aj[1] = add_f32(aj[1], g1, mjf); aj[2] = add_f32(aj[2], g2, mjf);
        }
    }

    /* 3b. pair forces over this walker's own points, after its springs, in the order
     *     gravity, coulomb, bounce.  Gravity / coulomb, for each pair i < j (gym/engine.py:128-147):
     *     r = max(norm(pos_i - pos_j) as float64, Config.r); f = -c * q_i * q_j / r**2 (Python floats:
     *     c, q = Config.g, m or Config.k, e); j.anti_forced(f, i) then i.anti_forced(f, j) (:69-76):
     *     force = -f * direction / distance, all float64 (f is a numpy float64 scalar: r came from
     *     .astype(float)); forced: a += force / m (float64, rounded to float32). */
    for (int pass = 0; pass < 2; pass++) {
        if (!(p->pair_mode & (1 << pass))) continue;
        const double cc = pass == 0 ? p->pair_g : p->pair_k;
        for (int i = m0; i < m1; i++)
            for (int j = i + 1; j < m1; j++) {
                const float *pi = pos + 3 * i, *pj = pos + 3 * j;
                double r = (double)np_norm3(pi[0] - pj[0], pi[1] - pj[1], pi[2] - pj[2]);
                if (CONFIG_R > r) r = CONFIG_R;
                const double qi = pass == 0 ? (double)b->m[i] : (b->charge ? b->charge[i] : p->pair_e);
                const double qj = pass == 0 ? (double)b->m[j] : (b->charge ? b->charge[j] : p->pair_e);
                const double f = ((-cc) * qi) * qj / (r * r);
                for (int c = 0; c < 3; c++) acc[3 * j + c] = add_f64(acc[3 * j + c], (-f) * (double)(pi[c] - pj[c]) / r, b->m[j]);
                for (int c = 0; c < 3; c++) acc[3 * i + c] = add_f64(acc[3 * i + c], (-f) * (double)(pj[c] - pi[c]) / r, b->m[i]);
            }
    }
    /*     Bounce: for s in registry order, for every other point i (gym/engine.py:114-125): if
     *     norm(s.pos - i.pos).astype(float) <= s.r + i.r: s.resilience(i, s.r + i.r, k / 2) (:78-102),
     *     a rigid spring of rest x = s.r + i.r (Python float, weakly cast to float32 in dx = current - x)
     *     and stiffness k/2 (float32 in f_size = -dx * k), applied to s then to i as in the spring pass.
     *     With a bounce_set, only the callers s (bit 0) bounce, each against `other` = the points with bit 1. */
    if (p->pair_mode & 4) {
        const float kb = (float)(p->bounce_k / 2);
        const uint8_t *bs = b->bounce_set;
        for (int s = m0; s < m1; s++) {
            if (bs && !(bs[s] & 1)) continue;
            for (int i = m0; i < m1; i++) {
                if (i == s || (bs && !(bs[i] & 2))) continue;
                const float *ps = pos + 3 * s, *pi = pos + 3 * i;
                const double x = b->radius[s] + b->radius[i];
                const float cur = np_norm3(ps[0] - pi[0], ps[1] - pi[1], ps[2] - pi[2]);
                if (!((double)cur <= x)) continue;
                const float dx = cur - (float)x;
                const float nf = -((-dx) * kb);
                double dist = (double)cur;
                if (CONFIG_R > dist) dist = CONFIG_R;
                for (int c = 0; c < 3; c++) acc[3 * s + c] = add_f64(acc[3 * s + c], (double)(nf * (pi[c] - ps[c])) / dist, b->m[s]);
                for (int c = 0; c < 3; c++) acc[3 * i + c] = add_f64(acc[3 * i + c], (double)(nf * (ps[c] - pi[c])) / dist, b->m[i]);
            }
        }
    }
    /*     G2 Point.gravity = gravity_vec (gym/optimized_engine.py:167-197; the performance_demo loop's N-body,
     *     gym/performance_demo.py:52-58): with >= 2 points every a is zeroed first (:174-175, discarding the
     *     springs above), then for each pair i < j: direction = p_j - p_i; distance = norm(direction), a numpy
     *     float32 (no .astype(float), :185-186); max(distance, Config.r); f = -Config.g * m_i * m_j / distance ** 2
     *     (:189: the Python-float numerator weakly cast to float32, distance ** 2 = libm powf); force = f *
     *     direction / distance (:192, float32); p_i.forced(force), p_j.forced(-force) (:193-194, float32 a += f/m).
     *     A clamped distance is the Python float Config.r: f and the division by it then take its float32 casts. */
    if ((p->pair_mode & 8) && m1 - m0 >= 2) {
        for (int q = m0; q < m1; q++) acc[3 * q] = acc[3 * q + 1] = acc[3 * q + 2] = 0.f;
        for (int i = m0; i < m1; i++)
            for (int j = i + 1; j < m1; j++) {
                const float *pi = pos + 3 * i, *pj = pos + 3 * j;
                const float d[3] = {pj[0] - pi[0], pj[1] - pi[1], pj[2] - pi[2]};
                const float dist = np_norm3(d[0], d[1], d[2]);
                const double num = (-p->pair_g * (double)b->m[i]) * (double)b->m[j];
                float f, dv;
                if (CONFIG_R > (double)dist) { f = (float)(num / (CONFIG_R * CONFIG_R)); dv = (float)CONFIG_R; }
                else { f = (float)num / powf(dist, 2.0f); dv = dist; }
                for (int c = 0; c < 3; c++) {
                    const float force = (f * d[c]) / dv;
                    acc[3 * i + c] = add_f32(acc[3 * i + c], force, b->m[i]);
                    acc[3 * j + c] = add_f32(acc[3 * j + c], -force, b->m[j]);
                }
            }
    }
    /*     Point.electrostatic (gym/engine.py:150-158) of every point, in registry order: for every other point i,
     *     r = max(norm(p_s - p_i) as float64, Config.r); f = -Config.k * e_s * e_i / r**2 (self's charge first);
     *     s.anti_forced(f, i) (:69-76): only s receives (-f) * (p_i - p_s) / r in float64, divided by m. */
    if (p->pair_mode & 16) {
        for (int s = m0; s < m1; s++)
            for (int i = m0; i < m1; i++) {
                if (i == s) continue;
                const float *ps = pos + 3 * s, *pi = pos + 3 * i;
                double r = (double)np_norm3(ps[0] - pi[0], ps[1] - pi[1], ps[2] - pi[2]);
                if (CONFIG_R > r) r = CONFIG_R;
                const double es = b->charge ? b->charge[s] : p->pair_e, ei = b->charge ? b->charge[i] : p->pair_e;
                const double f = ((-p->pair_k) * es) * ei / (r * r);
                for (int c = 0; c < 3; c++) acc[3 * s + c] = add_f64(acc[3 * s + c], (-f) * (double)(pi[c] - ps[c]) / r, b->m[s]);
            }
    }

    /* 4. env forces per mass (gym/env.py:31-41, gym/optimized_env.py:146-172), each one Point.forced
     *    with a float32 force: gravity, linear damp, then (in contact) ground spring, ground damp,
     *    friction |deep|*friction (optimized_env.py:168-172 form). */
    const float g = (float)(-p->g), dampk = (float)(-p->dampk), ground = (float)p->ground;
    const float gk = (float)(-p->groundk), gd = (float)(-p->grounddamp), fr = (float)p->friction;
    const float dt = (float)p->dt;
    for (int q = m0; q < m1; q++) {
        float *a = acc + 3 * q, *v = vel + 3 * q, *x = pos + 3 * q;
        const float mf = b->m[q];
        a[0] = add_f32(a[0], 0.f, mf); a[1] = add_f32(a[1], g, mf); a[2] = add_f32(a[2], 0.f, mf);
        a[0] = add_f32(a[0], dampk * v[0], mf);
        a[1] = add_f32(a[1], dampk * v[1], mf);
        a[2] = add_f32(a[2], dampk * v[2], mf);
        const float deep = x[1] - ground;
        const int hit = deep < 0.f;
        if (hit) {
            a[0] = add_f32(a[0], 0.f, mf); a[1] = add_f32(a[1], gk * deep, mf); a[2] = add_f32(a[2], 0.f, mf);
            a[0] = add_f32(a[0], 0.f, mf); a[1] = add_f32(a[1], gd * v[1], mf); a[2] = add_f32(a[2], 0.f, mf);
            const float ff = fabsf(deep) * fr;
            /* friction_mode 1: the G1 env's [v_x*deep*friction, 0, v_z*deep*friction] (gym/env.py:41) */
            const float fx = p->friction_mode ? (v[0] * deep) * fr : (-v[0]) * ff;
            const float fz = p->friction_mode ? (v[2] * deep) * fr : (-v[2]) * ff;
            a[0] = add_f32(a[0], fx, mf); a[1] = add_f32(a[1], 0.f, mf);
            a[2] = add_f32(a[2], fz, mf);
        }
        if (b->contact) b->contact[q] = (uint8_t)hit;   /* replaces color/r (optimized_env.py:155-175) */
        if (b->radius) b->radius[q] = hit ? 3.0 : 1.0;  /* p.r = 3 / p.r = 1 (optimized_env.py:156,175) */
        /* DingPoint (gym/optimized_engine.py:404-416): forced() is a no-op, so every force above left
         * its a at the zeros() of step 2; the env then integrates it with the base Point.run1. */
        if (b->pinned && b->pinned[q]) a[0] = a[1] = a[2] = 0.f;
        if (p->integrator == 2) {
            /* 5'. Point.run2 (gym/engine.py:180-190): pos += v*t + 0.5*a*t**2; v += a*t.  numpy order:
             *     (v*t) + ((0.5*a) * float32(t**2)), t**2 a Python float. */
            const float dt2 = (float)(p->dt * p->dt);
            for (int c = 0; c < 3; c++) x[c] = x[c] + (v[c] * dt + (0.5f * a[c]) * dt2);
            for (int c = 0; c < 3; c++) v[c] = v[c] + a[c] * dt;
        } else {
            /* 5. Point.run1 (gym/engine.py:168-178): v += a*t; pos += v*t; old_a = a; a = 0. */
            v[0] = v[0] + a[0] * dt; v[1] = v[1] + a[1] * dt; v[2] = v[2] + a[2] * dt;
            x[0] = x[0] + v[0] * dt; x[1] = x[1] + v[1] * dt; x[2] = x[2] + v[2] * dt;
        }
        /* acc now holds old_a (the acceleration used in this step) */
    }
    b->steps[w] += 1;                                    /* PhysicsEnv.step, optimized_env.py:84 */
}

/* Creature.getstat (gym/optimized_walker.py:129-162) + _get_reward/_is_done/_get_info/
 * _calculate_energy (gym/optimized_env.py:189-248) for one walker. */
static void walker_observe(const orc_batch *b, const orc_params *p, int w, const orc_out *o) {
    const int m0 = b->mass_off[w], M = b->mass_off[w + 1] - m0;
    const int u0 = b->muscle_off[w], A = b->muscle_off[w + 1] - u0;
    const float *pos = b->pos + 3 * m0, *vel = b->vel + 3 * m0, *acc = b->acc + 3 * m0;
    float ybuf[1024], nbuf[1024], kbuf[1024], pbuf[1024];
    const float *ys = pos + 1;
    if (o->obs) {
        float *ob = o->obs + (int64_t)w * o->obs_stride;
        const int d = p->in3d ? 3 : 2;
        float mid[3] = {0.f, 0.f, 0.f};
        if (p->midform) {
            for (int q = 0; q < M; q++) { mid[0] += pos[3 * q]; mid[1] += pos[3 * q + 1]; mid[2] += pos[3 * q + 2]; }
            /* midform 2 = G1 Creature.getstat (gym/walker.py:88-96): the mean is never taken */
            if (p->midform != 2) {
                const float fm = (float)M;
                mid[0] /= fm; mid[1] /= fm; mid[2] /= fm;
            }
        }
        const float pk = (float)p->pk, vk = (float)p->vk, ak = (float)p->ak, mk = (float)p->mk;
        int n = 0;
        for (int q = 0; q < M; q++) {
            for (int c = 0; c < d; c++) ob[n++] = p->midform ? (pos[3 * q + c] - mid[c]) * pk : pos[3 * q + c] * pk;
            for (int c = 0; c < d; c++) ob[n++] = vel[3 * q + c] * vk;
            for (int c = 0; c < d; c++) ob[n++] = acc[3 * q + c] * ak;
        }
        if (p->conmid) { ob[n++] = mid[0]; ob[n++] = mid[1]; ob[n++] = mid[2]; }
        for (int u = 0; u < A; u++) ob[n++] = b->mx[u0 + u] * mk;
        for (; n < o->obs_stride; n++) ob[n] = 0.f;
    }
    if (M > 1024) return;   /* reductions below use stack buffers; callers keep M <= 1024 */
    const float fM = (float)M;
    for (int q = 0; q < M; q++) {
        ybuf[q] = ys[3 * q];
        nbuf[q] = np_norm3(vel[3 * q], vel[3 * q + 1], vel[3 * q + 2]);
    }
    const float cy = pairwise(ybuf, M, 1) / fM;                       /* np.mean, :193 / :215 */
    const float ground = (float)p->ground;
    if (o->reward) {
        const float av = pairwise(nbuf, M, 1) / fM;                   /* :196 */
        const float vpen = (-av) * 0.1f;                              /* :197 */
        int hits = 0;
        for (int q = 0; q < M; q++) hits += (ys[3 * q] - ground < 0.f);   /* :200 */
        const float cpen = (float)(-(double)hits * 0.5);
        o->reward[w] = (cy + vpen) + cpen;                            /* :203 */
    }
    if (o->done) {
        int done = b->steps[w] >= p->max_steps;                      /* :210 */
        if (!done && cy < (float)(p->ground - 50.0)) done = 1;        /* :218 */
        if (!done && b->steps[w] > 100) {                             /* :222-224 */
            int all = 1;
            for (int q = 0; q < M; q++) all &= (nbuf[q] < 0.1f);
            done = all;
        }
        o->done[w] = (uint8_t)done;
    }
    if (o->centroid) {                                                /* :236, axis-0 mean: sequential */
        float s[3] = {0.f, 0.f, 0.f};
        for (int q = 0; q < M; q++) { s[0] += pos[3 * q]; s[1] += pos[3 * q + 1]; s[2] += pos[3 * q + 2]; }
        o->centroid[3 * w] = s[0] / fM; o->centroid[3 * w + 1] = s[1] / fM; o->centroid[3 * w + 2] = s[2] / fM;
    }
    if (o->energy) {                                                  /* :240-248 */
        for (int q = 0; q < M; q++) {
            const float mf = b->m[m0 + q];
            kbuf[q] = mf * powf(nbuf[q], 2.0f);   /* np.float32 ** 2 is libm powf (not x*x) */
            const float mg = (float)((double)mf * p->g);
            pbuf[q] = mg * (ys[3 * q] - ground);
        }
        const float ke = 0.5f * pairwise(kbuf, M, 1);
        const float pe = pairwise(pbuf, M, 1);
        o->energy[w] = ke + pe;
    }
    (void)acc;
}

int orc_step(const orc_batch *b, const orc_params *p, const float *action, int32_t action_cols,
             int32_t action_stride, const orc_out *o, int32_t n_threads) {
    if (!b || !p) return -1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(static) if (n_threads != 1)
#endif
    for (int w = 0; w < b->N; w++) {
        walker_step(b, p, w, action, action_cols, action_stride);
        if (o) walker_observe(b, p, w, o);
    }
    (void)n_threads;
    return 0;
}

int orc_observe(const orc_batch *b, const orc_params *p, const orc_out *o, int32_t n_threads) {
    if (!b || !p || !o) return -1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(static) if (n_threads != 1)
#endif
    for (int w = 0; w < b->N; w++) walker_observe(b, p, w, o);
    (void)n_threads;
    return 0;
}

int orc_reset(const orc_batch *b, const orc_params *p, const float *noise, int32_t n_threads) {
    if (!b || !p) return -1;
    (void)n_threads;
    /* PhysicsEnv.reset (gym/optimized_env.py:53-68): a = 0; v[0], v[1] (+ v[2] if in3d) += noise
     * (a Python float added to a float32 element: rounded to float32 first); steps = 0. */
    for (int w = 0; w < b->N; w++) {
        for (int q = b->mass_off[w]; q < b->mass_off[w + 1]; q++) {
            if (noise) {
                b->vel[3 * q] = b->vel[3 * q] + noise[3 * q];
                b->vel[3 * q + 1] = b->vel[3 * q + 1] + noise[3 * q + 1];
                if (p->in3d) b->vel[3 * q + 2] = b->vel[3 * q + 2] + noise[3 * q + 2];
            }
        }
        b->steps[w] = 0;
    }
    return 0;
}
