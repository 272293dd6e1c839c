/*
 * pt_oracle.h — CPU ORACLE for the MI355X path tracer.  TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference OptiX hot path (Damo12320/OptixPathtracer,
 * OptixPathtracer/source/Renderer/OptiX/devicePrograms.cu + the PBRT BSDF headers).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the
 * checker / the timed CPU baseline.  The product (optixpathtracer_amd/) never links it.
 *
 * Parity status: the reference cannot be compiled or run here (no nvcc/OptiX/NVIDIA GPU;
 * host-compiling its headers was denied by the environment).  This
 * restatement is therefore pinned only by the reference's own known answers
 * (UnitTests/SpherGeom_Test.cpp: CosTheta KAT + furnace bounds) and by the standard
 * TEA/LCG constants; everything else is "parity unpinned" against the OptiX original.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* material_mode: which BSDF pair the closest-hit program uses (devicePrograms.cu:303-341). */
enum {
    ORC_MAT_DEFAULT = 0,    /* rnd < metallic ? Conductor : GlossyDiffuse (active reference code) */
    ORC_MAT_LAMBERT = 1,    /* commented alternative, devicePrograms.cu:306/326 */
    ORC_MAT_CONDUCTOR = 2,  /* devicePrograms.cu:307/327 */
    ORC_MAT_DIELECTRIC = 3, /* devicePrograms.cu:304/324 */
    ORC_MAT_LAYERED = 4     /* devicePrograms.cu:305/325 */
};

/* BSDF model ids for the KAT entry points. */
enum { ORC_BSDF_LAMBERT = 0, ORC_BSDF_CONDUCTOR = 1, ORC_BSDF_DIELECTRIC = 2, ORC_BSDF_LAYERED = 3 };

typedef struct orc_mesh {
    const float* vertices;   /* n_vertices*3, object space (Mesh::vertecies) */
    const float* normals;    /* n_vertices*3 or NULL (Mesh::normal) */
    const int32_t* indices;  /* n_triangles*3 (Mesh::index) */
    int32_t n_vertices;
    int32_t n_triangles;
    float model[16];         /* glm column-major Mesh::GetModelMatrix() */
    float albedo[3];
    float metallic;
    float roughness;
    const float* texcoords;  /* n_vertices*2 or NULL (Mesh::texCoord; zeros when absent, Mesh.cpp:50-53) */
    int32_t albedo_tex;      /* -1 = none (Mesh.h:35-37) */
    int32_t normal_tex;
    int32_t metal_rough_tex;
} orc_mesh;

typedef struct orc_texture {  /* Texture.h:5-12: RGBA8, row 0 first as stored */
    const uint32_t* rgba8;
    int32_t width, height;
} orc_texture;

typedef struct orc_launch {  /* LaunchParams.h:9-28 */
    int32_t width, height;
    float cam_pos[3];
    float inv_view[16];
    float inv_proj[16];
    const float* lights;     /* n_lights * 6: position xyz, color rgb (LightsStruct.h:6-10) */
    int32_t n_lights;
    int32_t max_bounces;
    int32_t material_mode;
} orc_launch;

typedef struct orc_scene orc_scene;

/* --- RNG (random.h:34-69) --- */
uint32_t orc_tea16(uint32_t v0, uint32_t v1);
/* The path's transcendentals (shared fixed polynomials, see pt_oracle.c): fn 0 = sin, 1 = cos
 * (|x| <= 2^15), 2 = exp (x <= 0), 3 = x^2.4 (x in (0, 1]). */
void orc_math_eval(int32_t fn, const float* x, float* out, int32_t n);
void orc_rnd_seq(uint32_t seed, int32_t n, float* out, uint32_t* seed_out);
uint32_t orc_f2u_sat(float f);

/* --- BSDF KATs (shading space, N = +z) --- */
/* out: color[3], pdf, direction[3], flags (bit0 refl, bit1 trans, bit2 specular, bit3 glossy) */
int32_t orc_bsdf_sample(int32_t model, uint32_t* seed, const float albedo[3], float roughness,
                        const float wo[3], float out[8]);
void orc_bsdf_eval(int32_t model, uint32_t* seed, const float albedo[3], float roughness,
                   const float wo[3], const float wi[3], float out[3]);
float orc_bsdf_pdf(int32_t model, float roughness, const float wo[3], const float wi[3]);
void orc_bsdf_sample_n(int32_t model, uint32_t* seed, const float albedo[3], float roughness, const float wo[3],
                       int32_t n, float* out8, int32_t* ok);
void orc_bsdf_pdf_n(int32_t model, float roughness, const float wo[3], const float* wi3, int32_t n, float* out);
/* reference unit-test known answers (UnitTests/SpherGeom_Test.cpp) */
float orc_cos_theta(const float w[3]);
void orc_furnace(int32_t model, uint32_t* seed, const float albedo[3], float roughness, const float wo[3],
                 int32_t n, float out[3]);

/* --- camera (Camera.cpp:37-70, GlmHelperMethods.cpp:4-10, OptixRenderer.cpp:662-668) --- */
void orc_camera_from_blender(const float blender_pos[3], const float blender_rot_deg[3],
                             float fov_deg, int32_t width, int32_t height,
                             float pos[3], float inv_view[16], float inv_proj[16]);
void orc_camera_ray(const orc_launch* lp, int32_t x, int32_t y, float origin[3], float dir[3]);

/* --- scene + traversal --- */
orc_scene* orc_scene_create(const orc_mesh* meshes, int32_t n_meshes, const orc_texture* textures,
                            int32_t n_textures);
/* tex2D<float4> of CreateTextures' texture objects (OptixRenderer.cpp:562-612): bilinear,
 * wrap, normalized coordinates, normalized-float read; sRGB decode optional (SRGB8ToLinear). */
void orc_tex_sample(const orc_texture* t, float x, float y, int32_t srgb, float out[4]);
void orc_scene_destroy(orc_scene* s);
int32_t orc_scene_triangles(const orc_scene* s);
/* returns global primitive index (meshes concatenated) or -1 */
int32_t orc_trace_closest(const orc_scene* s, const float o[3], const float d[3], float tmin,
                          float tmax, float* t, float* u, float* v, int32_t* backface);
int32_t orc_trace_any(const orc_scene* s, const float o[3], const float d[3], float tmin, float tmax);
/* Diagnostic: repeat every closest-hit trace without culling by the running best t and count
 * disagreements (out[0] traces, out[1] mismatches; first[16] = the first mismatching ray:
 * o, d, tmin, tmax, prim, t, prim_exhaustive, t_exhaustive, u, v, u_exh, v_exh). */
void orc_set_cull_check(int32_t on);
void orc_cull_check_stats(uint64_t out[2], float first[16]);

/* --- the hot path: per-pixel sum of radiance over frame ids [first_frame, first_frame+n_frames)
 *     for pixels x in [x0,x1), y in [y0,y1); sum_rgb is the full W*H*3 buffer (row 0 = bottom).
 *     The sum is ADDED into sum_rgb (sequential fp32 adds in frame order). --- */
void orc_render(const orc_scene* s, const orc_launch* lp, uint32_t first_frame, uint32_t n_frames,
                int32_t x0, int32_t y0, int32_t x1, int32_t y1, float* sum_rgb, int32_t n_threads,
                uint64_t* segments_out);
/* one path (debug / per-sample parity) */
void orc_sample_path(const orc_scene* s, const orc_launch* lp, int32_t x, int32_t y, uint32_t frame,
                     float out_rgb[3], int32_t* segments);
/* The reference's debug pixel (devicePrograms.cu:637-644, printed at :428-437) as data: one path,
 * ORC_DEBUG_FLOATS per shaded bounce (layout of ptamd.h pt_debug_bounce: bounce and prim as int32
 * bits, position, albedo, shading normal, geometry normal, roughness, metallic, throughput
 * entering the bounce, radiance before its NEE); returns the number of bounces recorded. */
#define ORC_DEBUG_FLOATS 22
int32_t orc_sample_path_debug(const orc_scene* s, const orc_launch* lp, int32_t x, int32_t y, uint32_t frame,
                              float* records, int32_t max_bounces, float out_rgb[3]);

#ifdef __cplusplus
}
#endif
#endif
