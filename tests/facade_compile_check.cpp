// Compile-and-link check of include/OptixRenderer.hpp against stand-in types shaped like
// the reference's Model / Mesh / Camera / PointLight / glm (the reference sources are not
// compiled; these minimal structs only mimic the member names the facade uses).  Without a
// GPU the constructor must throw (pt_create fails loudly); with one it renders 1 spp.
#include <cstdio>
#include <memory>
#include <vector>

#include <cstring>

#include "OptixRenderer.hpp"

namespace stand_in {
struct vec2 { float x, y; };
struct vec3 { float x, y, z; };
struct ivec2 { int x, y; };
struct ivec3 { int x, y, z; };
struct mat4 {
    float c[4][4];
    const float* operator[](int i) const { return c[i]; }
};
struct Mesh {
    std::vector<vec3> vertecies, normal;
    std::vector<vec2> texCoord;
    std::vector<ivec3> index;
    vec3 albedo{0.5f, 0.5f, 0.5f};
    float metallic = 0.0f, roughness = 0.5f;
    int albedoTex = -1, normalTex = -1, metalRoughTex = -1;
    mat4 GetModelMatrix() const {
        mat4 m{};
        for (int i = 0; i < 4; ++i) m.c[i][i] = 1.0f;
        return m;
    }
};
struct Texture {
    uint32_t* pixel = nullptr;
    ivec2 resolution{-1, -1};
};
struct Model {
    std::vector<std::unique_ptr<Mesh>> meshes;
    std::vector<std::unique_ptr<Texture>> textures;
};
struct PointLight {
    vec3 position, color;
};
struct Camera {
    vec3 position{0, 0, 3};
    mat4 GetViewMatrix() const {
        mat4 m{};
        for (int i = 0; i < 4; ++i) m.c[i][i] = 1.0f;
        m.c[3][2] = -3.0f;
        return m;
    }
    mat4 GetProjectionMatrix(float aspect) const {
        mat4 m{};
        m.c[0][0] = 1.0f / aspect;
        m.c[1][1] = 1.0f;
        m.c[2][2] = -1.002f;
        m.c[2][3] = -1.0f;
        m.c[3][2] = -0.2002f;
        return m;
    }
};
}  // namespace stand_in

int main() {
    using namespace stand_in;
    Model model;
    auto m = std::make_unique<Mesh>();
    m->vertecies = {{-1, -1, 0}, {1, -1, 0}, {0, 1, 0}};
    m->normal = {{0, 0, 1}, {0, 0, 1}, {0, 0, 1}};
    m->index = {{0, 1, 2}};
    model.meshes.push_back(std::move(m));
    try {
        ptamd::OptixRendererT<Model> r("ignored.ptx", &model, PT_MAT_LAMBERT);
        ivec2 size{8, 8};
        r.Resize(size);
        Camera cam;
        r.SetCamera(&cam);
        std::vector<PointLight> lights = {{{0, 0, 2}, {1, 1, 1}}};
        r.SetLights(&lights);
        r.SetMaxBounces(2);
        std::vector<vec3> px(64);
        r.Render(px.data());
        float mx = 0.0f;
        for (const auto& v : px) mx = v.x > mx ? v.x : mx;
        std::printf("rendered max=%g\n", mx);
        std::vector<vec3> mean(64);
        r.RenderAccumulate(4, 1, mean.data());  // extension beyond the reference's six methods
        float mm = 0.0f;
        for (const auto& v : mean) mm = v.x > mm ? v.x : mm;
        std::printf("accumulated max=%g\n", mm);
        // multi-GPU inside the library: the same image from a renderer over a device list (one
        // RCCL communicator; one device here, so the reduce must return the image bit for bit)
        ptamd::OptixRendererT<Model> rm("ignored.ptx", &model, PT_MAT_LAMBERT, 0, PT_KERNEL_AUTO, {0});
        rm.Resize(size);
        rm.SetCamera(&cam);
        rm.SetLights(&lights);
        rm.SetMaxBounces(2);
        std::vector<vec3> mean_multi(64);
        rm.RenderAccumulate(4, 1, mean_multi.data());
        const bool same = std::memcmp(mean.data(), mean_multi.data(), sizeof(vec3) * mean.size()) == 0;
        std::printf("device-list image identical=%d\n", same ? 1 : 0);
        return (mx > 0.0f && mm > 0.0f && same) ? 0 : 3;
    } catch (const std::exception& e) {
        std::printf("threw: %s\n", e.what());
        return 2;
    }
}
