/* Host-side AddressSanitizer driver for libwalker_hip's CPU code (tests/test_host_asan.py): the wave / workgroup
 * planners on seeded ragged batches in exactly-sized buffers, their error paths, launch geometry and argument
 * validation.  Nothing here launches a kernel or touches a GPU. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "walker_hip.h"

static int32_t *offsets(int N, const int *sizes) {
    int32_t *o = (int32_t *)malloc(sizeof(int32_t) * (N + 1));
    o[0] = 0;
    for (int w = 0; w < N; w++) o[w + 1] = o[w] + sizes[w];
    return o;
}

int main(void) {
    int bad = 0;
    srand(7);
    for (int rep = 0; rep < 20; rep++) {
        const int N = 1 + rand() % 3000;
        int *Ms = (int *)malloc(sizeof(int) * N), *Ks = (int *)malloc(sizeof(int) * N), *As = (int *)malloc(sizeof(int) * N);
        for (int w = 0; w < N; w++) { Ms[w] = 1 + rand() % 64; Ks[w] = rand() % (Ms[w] + 1); As[w] = Ks[w] / 5; }
        int32_t *mo = offsets(N, Ms), *eo = offsets(N, Ks), *uo = offsets(N, As);
        int32_t *plan = (int32_t *)malloc(sizeof(int32_t) * (N + 1));
        const int nt = wg_plan_waves(mo, eo, uo, N, plan, N);          /* capacity N tiles: plan has N + 1 slots */
        const int nb = wg_plan_ragged(mo, eo, uo, N, plan, N);
        if (nt <= 0 || nb <= 0 || plan[0] != 0) { printf("rep %d: plans %d %d\n", rep, nt, nb); bad = 1; }
        if (wg_plan_waves(mo, eo, uo, N, plan, 1) != WG_ERANGE && N > 64) { printf("rep %d: no ERANGE\n", rep); bad = 1; }
        free(Ms); free(Ks); free(As); free(mo); free(eo); free(uo); free(plan);
    }
    int big[1] = {65}, k[1] = {4}, a[1] = {0};
    int32_t *mo = offsets(1, big), *eo = offsets(1, k), *uo = offsets(1, a), plan[2];
    if (wg_plan_waves(mo, eo, uo, 1, plan, 1) != WG_EINVAL) { printf("no EINVAL for M=65\n"); bad = 1; }
    if (wg_plan_waves(NULL, eo, uo, 1, plan, 1) != WG_EINVAL) { printf("no EINVAL for NULL\n"); bad = 1; }
    free(mo); free(eo); free(uo);
    for (int M = 1; M <= 70; M++)
        for (int K = 0; K <= 600; K += 7) (void)wg_wave_edge_passes(M, K);
    wg_batch b;
    memset(&b, 0, sizeof b);
    b.N = 65536; b.M = 16; b.K = 40; b.A = 8;
    float dummy[4];
    b.pos = b.vel = b.acc = dummy; b.mass = dummy; b.muscle_x = dummy;
    b.edges = (const wg_edge *)dummy; b.inc = (const uint16_t *)dummy; b.inc_off = (const uint16_t *)dummy;
    b.steps = (int32_t *)dummy;
    wg_launch_info info;
    if (wg_launch_geometry(&b, &info) != 0 || info.blocks != 4096) { printf("geometry %d\n", info.blocks); bad = 1; }
    if (wg_step(&b, NULL, NULL, 0, 0, 0, NULL, 1, NULL, 0, NULL) != WG_EINVAL) { printf("null params accepted\n"); bad = 1; }
    if (strlen(wg_last_error()) == 0) { printf("no error message\n"); bad = 1; }
    printf(bad ? "FAILED\n" : "host asan ok\n");
    return bad;
}
