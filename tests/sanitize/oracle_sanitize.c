/* The oracle (oracle/oracle.c, test infrastructure) under ASan + UBSan: the reference world, a frame of
   castRayFromCam rays, AO, shading in both liquid modes, deleteBlock with the reference's shift defect,
   and the collapsed terrain builder.  Built and run by tests/test_sanitizers.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct otree otree;
otree* orc_tree_new(int levels);
void orc_tree_free(otree* t);
void orc_init_tetra_hexa_tree(otree* t);
void orc_gen_world(otree* t, int w, int l);
int orc_build_terrain_collapsed(otree* t, const int32_t* h, int W, int L);
void orc_heights(int W, int L, int32_t* out, int nthreads);
void orc_normalize(const float* v, float* o);
void orc_proj_plane(int W, int H, float* ppx, float* ppy);
int orc_cast_frame(const otree* t, const float* org, const float* cam, float ppx, float ppy, int W, int H, int steps, const int64_t* pix,
                   int64_t n, int nthreads, int32_t* pos, int32_t* last, int32_t* stp, int32_t* hit, double* tt, uint64_t* col,
                   uint32_t* fl, int32_t* ax, uint64_t* dda);
void orc_cast_frame_ao(const otree* t, const float* org, const float* cam, float ppx, float ppy, int W, int H, int steps, int n_ao,
                       int ao_steps, const int64_t* pix, int64_t n, int nthreads, uint8_t* ao, int32_t* hit);
void orc_shade_frame(const otree* t, const float* org, const float* cam, float ppx, float ppy, int W, int H, int steps, const float* sun,
                     const int32_t* look, int shadow_steps, const int64_t* pix, int64_t n, int nthreads, float* rgba, int liquid, float time);
int orc_delete_block(otree* t, int x, int y, int z, int level, int ref_shift, uint32_t* f, uint64_t* c, float* m);
uint64_t orc_frame_entries_ao(const otree* t, const float* org, const float* cam, float ppx, float ppy, int W, int H, int steps, int n_ao,
                              int ao_steps, const int64_t* pix, int64_t n, int nthreads);

int main(void) {
    const int W = 96, H = 64, N = W * H;
    otree* t = orc_tree_new(5);
    orc_init_tetra_hexa_tree(t);
    orc_gen_world(t, 200, 200);
    float cam[3], d[3] = {1.0f, -0.45f, 1.0f}, org[3] = {4.0f, 90.0f, 4.0f}, sunv[3] = {2.0f, 1.0f, 4.0f}, sun[3], ppx, ppy;
    orc_normalize(d, cam);
    orc_normalize(sunv, sun);
    orc_proj_plane(W, H, &ppx, &ppy);
    int32_t *pos = malloc(12 * N), *last = malloc(12 * N), *stp = malloc(4 * N), *hit = malloc(4 * N), *ax = malloc(4 * N);
    double* tt = malloc(8 * N);
    uint64_t *col = malloc(8 * N), dda = 0;
    uint32_t* fl = malloc(4 * N);
    uint8_t* ao = malloc(N);
    float* rgba = malloc(16 * N);
    if (orc_cast_frame(t, org, cam, ppx, ppy, W, H, 300, NULL, N, 2, pos, last, stp, hit, tt, col, fl, ax, &dda)) return 1;
    orc_cast_frame_ao(t, org, cam, ppx, ppy, W, H, 300, 16, 5, NULL, N, 2, ao, hit);
    orc_shade_frame(t, org, cam, ppx, ppy, W, H, 300, sun, NULL, 75, NULL, N, 2, rgba, 0, 0.0f);
    orc_shade_frame(t, org, cam, ppx, ppy, W, H, 300, sun, NULL, 75, NULL, N, 2, rgba, 1, 1.5f);
    (void)orc_frame_entries_ao(t, org, cam, ppx, ppy, W, H, 300, 16, 5, NULL, N, 2);
    uint32_t f;
    uint64_t c;
    float m;
    for (int i = 0; i < 64; i++) orc_delete_block(t, 10 + i, 30, 40 + (i & 7), 6, i & 1, &f, &c, &m);
    orc_tree_free(t);
    int32_t* hg = malloc(4 * 256 * 256);
    orc_heights(256, 256, hg, 2);
    otree* u = orc_tree_new(5);
    if (orc_build_terrain_collapsed(u, hg, 256, 256)) return 1;
    orc_shade_frame(u, org, cam, ppx, ppy, W, H, 2000, sun, NULL, 75, NULL, N, 2, rgba, 1, 0.25f);
    orc_tree_free(u);
    free(hg); free(pos); free(last); free(stp); free(hit); free(ax); free(tt); free(col); free(fl); free(ao); free(rgba);
    printf("oracle sanitize ok\n");
    return 0;
}
