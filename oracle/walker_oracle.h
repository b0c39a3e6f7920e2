/* walker_oracle.h — CPU restatement of the reference walker step (TEST INFRASTRUCTURE ONLY).
 *
 * This is the checker, never the product: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  See walker_oracle.c for the per-line reference citations.
 * Layout: flat CSR over walkers (mass_off/edge_off/muscle_off, N+1 entries each); walker-local
 * edge endpoints; muscles are the first (muscle_off[w+1]-muscle_off[w]) edges of walker w.
 */
#ifndef WALKER_ORACLE_H
#define WALKER_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_params {
    double g, dampk, ground, groundk, grounddamp, friction, dt;
    double pk, vk, ak, mk;
    int32_t in3d, max_steps, midform, conmid;
    int32_t spring_mode;   /* 0 = engine.py resilience + G2 damping; 1 = G2 optimized_walker as written;
                              2 = the G3 engine (optimized_walker/core.py springs, env.py update_physics) */
    int32_t action_mode;   /* 0 = Muscle.act (continuous); 1 = Muscle.actdisp (discrete) */
    int32_t integrator;    /* 0/1 = Point.run1 (gym/engine.py:168-178); 2 = Point.run2 (:180-190) */
    int32_t pair_mode;     /* bitmask, per walker after the springs, in this order: 1 = Point.gravity
                              (gym/engine.py:128-137), 2 = Point.coulomb (:139-147), 4 = Point.bounce
                              of every caller in registry order against its `other` set (:114-125) */
    double pair_g;         /* Config.g of the gravity pass (gym/engine.py:12) */
    double pair_k;         /* Config.k of the coulomb pass (gym/engine.py:11) */
    double pair_e;         /* Point.e when charge == NULL (Config.e, gym/engine.py:10) */
    double bounce_k;       /* Point.bounce(k) (gym/engine.py:114, default 100) */
    /* spring_mode 2: the G3 engine, Environment.update_physics (gym/optimized_walker/env.py:135-184) */
    double g3_gravity[3];  /* Environment.gravity (default (0, -9.8, 0)) */
    double g3_damping, g3_air, g3_ground_level, g3_restitution, g3_friction;
    int32_t g3_ground;     /* Environment.ground: the position-clamp ground is on */
    int32_t friction_mode; /* ground friction: 0 = [-v_x*(|deep|*friction), 0, -v_z*(...)] (gym/optimized_env.py:
                              168-172); 1 = [v_x*deep*friction, 0, v_z*deep*friction] (the G1 env, gym/env.py:41) */
} orc_params;

typedef struct orc_batch {
    int32_t N;
    const int32_t *mass_off, *edge_off, *muscle_off;
    float *pos, *vel, *acc;          /* [P*3] */
    const float *m;                  /* [P]   */
    const int32_t *ei, *ej;          /* [E] walker-local */
    const float *rest, *k, *c;       /* [E]; rest of a muscle edge = its originx */
    const uint8_t *flags;            /* [E] bit0 string (may be NULL) */
    float *mx;                       /* [U] muscle rest length state */
    const float *minl, *maxl, *stride; /* [U] */
    int32_t *steps;                  /* [N] */
    uint8_t *contact;                /* [P] (may be NULL) */
    const uint8_t *pinned;           /* [P] 1 = DingPoint, forced() a no-op (may be NULL) */
    const double *charge;            /* [P] Point.e (Python floats); NULL = pair_e for every point */
    double *radius;                  /* [P] Point.r (Python floats), read by bounce; the env pass sets
                                        3 on contact, 1 otherwise (optimized_env.py:156,175); may be NULL
                                        unless pair_mode & 4 */
    const uint8_t *bounce_set;       /* [P] Point.bounce(k, other=<list>) (gym/engine.py:114-125): bit 0 = the point
                                        calls bounce (callers in registry order), bit 1 = the point is in `other`
                                        (the list in registry order); NULL = every point, other="*" */
} orc_batch;

typedef struct orc_out {
    float *obs; int32_t obs_stride;  /* [N*obs_stride] (may be NULL) */
    float *reward; uint8_t *done; float *centroid; float *energy;  /* each may be NULL */
} orc_out;

int orc_abi_version(void);
/* One env step for every walker: act -> springs -> env forces -> run1 -> observe. */
int orc_step(const orc_batch *b, const orc_params *p, const float *action, int32_t action_cols,
             int32_t action_stride, const orc_out *o, int32_t n_threads);
/* Observation / reward / done / info for the current state (reset path; no physics). */
int orc_observe(const orc_batch *b, const orc_params *p, const orc_out *o, int32_t n_threads);
/* PhysicsEnv.reset: a = 0, v += noise (x,y; z if in3d), steps = 0. noise [P*3] (may be NULL). */
int orc_reset(const orc_batch *b, const orc_params *p, const float *noise, int32_t n_threads);
/* numpy float32 helpers exported for unit tests */
float orc_np_norm3(const float *v);
float orc_np_pairwise_sum(const float *a, int64_t n, int64_t stride);

#ifdef __cplusplus
}
#endif
#endif
