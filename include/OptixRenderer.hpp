// OptixRenderer.hpp — header-only C++ drop-in for the reference's
// Renderer/OptiX/OptixRenderer.h (Damo12320/OptixPathtracer), forwarding to the C ABI of
// libptamd.so (include/ptamd.h).
//
// The reference's callers (Renderer/OptixView.cpp:89-255, main.cpp:95-113) use exactly
//   OptixRenderer(const std::string& ptxPath, Model* model);      // OptixRenderer.h:67
//   void Resize(glm::ivec2& newSize);                              // :70
//   void Render(glm::vec3 h_pixels[]);                             // :72
//   void SetCamera(Camera* camera);                                // :74
//   void SetLights(std::vector<PointLight>* lights);               // :75
//   void SetMaxBounces(int maxBounces);                            // :76
//   Model* model;                                                  // :64
// This header keeps those names and argument meanings.  It is written against the
// reference's types by duck typing (templates), so it needs neither glm nor the
// reference's headers to compile on its own; in the reference build, Model/Mesh/Camera/
// PointLight/glm are the reference's own.  ptxPath is accepted and ignored (no PTX on
// gfx950).  Errors throw std::runtime_error, as the reference's CUDA_CHECK does
// (3rdParty/OptixSample/optix7.h:26-36).
#pragma once

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ptamd.h"

namespace ptamd {

inline void check(int status, const char* what) {
    if (status != PT_OK) throw std::runtime_error(std::string(what) + ": " + pt_last_error());
}

template <class ModelT>
class OptixRendererT {
   public:
    ModelT* model;

    // devices: empty = the single `device`; otherwise every listed device renders a share of
    // the frame ids of RenderFrames / RenderAccumulate and RCCL sums the shares (pt_options.n_devices).
    OptixRendererT(const std::string& /*ptxPath*/, ModelT* m, int material_mode = PT_MAT_DEFAULT, int device = 0,
                   int kernel = PT_KERNEL_AUTO, const std::vector<int32_t>& devices = {})
        : model(m) {
        // Model::meshes (ModelLoading/Model.h:5-8) -> pt_mesh views (deep-copied by pt_create)
        std::vector<pt_mesh> meshes;
        std::vector<std::vector<int32_t>> idx;  // glm::ivec3 -> int32 triplets
        meshes.reserve(m->meshes.size());
        idx.reserve(m->meshes.size());
        for (auto& up : m->meshes) {
            auto& me = *up;
            pt_mesh pm;
            std::memset(&pm, 0, sizeof pm);
            pm.vertices = reinterpret_cast<const float*>(me.vertecies.data());
            pm.normals = me.normal.empty() ? nullptr : reinterpret_cast<const float*>(me.normal.data());
            pm.texcoords = me.texCoord.empty() ? nullptr : reinterpret_cast<const float*>(me.texCoord.data());
            idx.emplace_back();
            idx.back().reserve(me.index.size() * 3);
            for (auto& t : me.index) {
                idx.back().push_back((int32_t)t.x);
                idx.back().push_back((int32_t)t.y);
                idx.back().push_back((int32_t)t.z);
            }
            pm.indices = idx.back().data();
            pm.n_vertices = (int32_t)me.vertecies.size();
            pm.n_triangles = (int32_t)me.index.size();
            auto mm = me.GetModelMatrix();  // column-major glm::mat4 (Mesh.cpp:6-22)
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) pm.model_matrix[c * 4 + r] = mm[c][r];
            pm.albedo[0] = me.albedo.x;
            pm.albedo[1] = me.albedo.y;
            pm.albedo[2] = me.albedo.z;
            pm.metallic = me.metallic;
            pm.roughness = me.roughness;
            pm.albedo_tex = me.albedoTex;
            pm.normal_tex = me.normalTex;
            pm.metal_rough_tex = me.metalRoughTex;
            meshes.push_back(pm);
        }
        // Model::textures (Texture.h:5-12: uint32_t* pixel RGBA8, ivec2 resolution)
        std::vector<pt_texture> textures;
        for (auto& tp : m->textures) {
            pt_texture t;
            t.rgba8 = tp->pixel;
            t.width = (int32_t)tp->resolution.x;
            t.height = (int32_t)tp->resolution.y;
            textures.push_back(t);
        }
        pt_scene sc;
        std::memset(&sc, 0, sizeof sc);
        sc.meshes = meshes.data();
        sc.n_meshes = (int32_t)meshes.size();
        sc.textures = textures.empty() ? nullptr : textures.data();
        sc.n_textures = (int32_t)textures.size();
        pt_options opt;
        std::memset(&opt, 0, sizeof opt);
        opt.device = device;
        opt.material_mode = material_mode;
        opt.kernel = kernel;
        opt.n_devices = (int32_t)devices.size();
        opt.device_list = devices.empty() ? nullptr : devices.data();
        check(pt_create(&sc, &opt, &r_), "pt_create");
    }
    ~OptixRendererT() { pt_destroy(r_); }
    OptixRendererT(const OptixRendererT&) = delete;
    OptixRendererT& operator=(const OptixRendererT&) = delete;

    template <class IVec2>
    void Resize(IVec2& newSize) {  // OptixRenderer.cpp:649-660
        check(pt_resize(r_, (int32_t)newSize.x, (int32_t)newSize.y), "pt_resize");
        if (newSize.x != 0 && newSize.y != 0) {
            w_ = newSize.x;
            h_ = newSize.y;
        }
    }

    template <class Vec3>
    void Render(Vec3 h_pixels[]) {  // OptixRenderer.cpp:617-647 (1 spp, frame.id++)
        static_assert(sizeof(Vec3) == 3 * sizeof(float), "h_pixels must be glm::vec3-like");
        check(pt_render(r_, reinterpret_cast<float*>(h_pixels)), "pt_render");
    }

    template <class CameraT>
    void SetCamera(CameraT* camera) {  // OptixRenderer.cpp:662-668
        const float aspect = w_ / float(h_);
        auto iv = inverse4(camera->GetViewMatrix());
        auto ip = inverse4(camera->GetProjectionMatrix(aspect));
        float pos[3] = {camera->position.x, camera->position.y, camera->position.z};
        check(pt_set_camera(r_, pos, iv.m, ip.m), "pt_set_camera");
    }

    template <class PointLightT>
    void SetLights(std::vector<PointLightT>* lights) {  // OptixRenderer.cpp:670-675
        std::vector<pt_point_light> pl(lights->size());
        for (size_t i = 0; i < lights->size(); ++i) {
            const auto& l = (*lights)[i];
            pl[i] = pt_point_light{{l.position.x, l.position.y, l.position.z}, {l.color.x, l.color.y, l.color.z}};
        }
        check(pt_set_lights(r_, pl.data(), (int32_t)pl.size()), "pt_set_lights");
    }

    void SetMaxBounces(int maxBounces) { check(pt_set_max_bounces(r_, maxBounces), "pt_set_max_bounces"); }

    // --- beyond the reference: device-resident accumulation (replaces OptixView's GL blend)
    void RenderFrames(uint32_t first_frame_id, uint32_t n) {
        check(pt_render_frames(r_, first_frame_id, n), "pt_render_frames");
    }
    void ClearAccumulation() { check(pt_accum_clear(r_), "pt_accum_clear"); }
    template <class Vec3>
    void DownloadMean(Vec3 h_pixels[], uint32_t spp) {
        check(pt_accum_download(r_, reinterpret_cast<float*>(h_pixels), 1.0f / (float)spp), "pt_accum_download");
    }
    // Whole image in one call: spp frames from first_frame_id, mean to h_pixels (W*H vec3).
    template <class Vec3>
    void RenderAccumulate(uint32_t spp, uint32_t first_frame_id, Vec3 h_pixels[]) {
        check(pt_render_accumulate(r_, spp, first_frame_id, reinterpret_cast<float*>(h_pixels)),
              "pt_render_accumulate");
    }
    pt_renderer* handle() { return r_; }

   private:
    struct M4 {
        float m[16];
    };
    // glm::inverse(mat4) (detail/func_matrix.inl compute_inverse<4,4>), same rounding order.
    template <class Mat4>
    static M4 inverse4(const Mat4& g) {
        float m[16];
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) m[c * 4 + r] = g[c][r];
        auto M = [&](int c, int r) { return m[c * 4 + r]; };
        float C00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3), C02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
        float C03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3), C04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
        float C06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3), C07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
        float C08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2), C10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
        float C11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2), C12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
        float C14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3), C15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
        float C16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2), C18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
        float C19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2), C20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
        float C22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1), C23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
        const float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
        const float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
        const float V0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)}, V1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
        const float V2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)}, V3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
        const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
        float I0[4], I1[4], I2[4], I3[4];
        for (int i = 0; i < 4; ++i) {
            I0[i] = (V1[i] * F0[i] - V2[i] * F1[i] + V3[i] * F2[i]) * SA[i];
            I1[i] = (V0[i] * F0[i] - V2[i] * F3[i] + V3[i] * F4[i]) * SB[i];
            I2[i] = (V0[i] * F1[i] - V1[i] * F3[i] + V3[i] * F5[i]) * SA[i];
            I3[i] = (V0[i] * F2[i] - V1[i] * F4[i] + V2[i] * F5[i]) * SB[i];
        }
        float d0 = M(0, 0) * I0[0], d1 = M(0, 1) * I1[0], d2 = M(0, 2) * I2[0], d3 = M(0, 3) * I3[0];
        float one = 1.0f / ((d0 + d1) + (d2 + d3));
        M4 out;
        for (int i = 0; i < 4; ++i) {
            out.m[i] = I0[i] * one;
            out.m[4 + i] = I1[i] * one;
            out.m[8 + i] = I2[i] * one;
            out.m[12 + i] = I3[i] * one;
        }
        return out;
    }

    pt_renderer* r_ = nullptr;
    int w_ = 0, h_ = 0;
};

}  // namespace ptamd
