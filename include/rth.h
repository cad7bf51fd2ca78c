/*
 * rth.h — C-ABI of the host scene front-end (librth.so), the part of RTBase that stays on the
 * CPU above the rtg boundary:
 *
 *   loadScene / loadInstance        RTBase/SceneLoader.h:104-291  -> rth_load_scene()
 *   GEMScene / GEMModelLoader       RTBase/GEMLoader.h:218-750    (scene.json + .gem parsing)
 *   Texture::load                   RTBase/Imaging.h:32-71        (PNG / Radiance .hdr decode)
 *   Scene::init / Scene::build      RTBase/Scene.h:82-106,142-160 (BVH build, light list)
 *   Film::save                      RTBase/Imaging.h:262-271      -> rth_save_hdr()
 *   Film::tonemap + savePNG         RTBase/Imaging.h:233-242, Renderer.h:895-898 -> rth_tonemap(), rth_save_png()
 *
 * It produces the flattened rtg_scene_desc consumed by rtg_create (include/rtg.h).
 */
#ifndef RTH_H
#define RTH_H

#include "rtg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rth_scene rth_scene;

typedef struct rth_load_options {
    int32_t width;          /* >0: override scene.json "width" before P is built (0 = keep)   */
    int32_t height;         /* >0: override scene.json "height" before P is built (0 = keep)  */
    int32_t skip_missing;   /* 1: drop instances whose .gem or reflectance file is missing    */
                            /*    (the "_f" filtered variants); 0: error    */
    int32_t bvh_threads;    /* host threads for the BVH build (0 = hardware concurrency)      */
    const char* envmap;     /* non-NULL: override scene.json "envmap" (file in the scene dir) */
} rth_load_options;

typedef struct rth_scene_info {
    uint32_t n_tris, n_nodes, n_materials, n_textures, n_lights, bvh_depth;
    int32_t width, height;
    int32_t env_in_lights;
    uint32_t dropped_instances;   /* instances skipped by skip_missing                      */
    double load_ms, bvh_ms;       /* wall time of parsing+transform and of Scene::build     */
    float bounds_min[3], bounds_max[3];
} rth_scene_info;

const char* rth_last_error(void);
/* Hash of the sources, headers and compile flags this library was built from (build.py). */
const char* rth_build_id(void);

int  rth_load_scene(const char* scene_dir, const rth_load_options* opts, rth_scene** out);
void rth_free_scene(rth_scene* s);
const rtg_scene_desc* rth_scene_desc(const rth_scene* s);
int  rth_scene_get_info(const rth_scene* s, rth_scene_info* out);
/* Index (pre-build load order) of each post-build triangle: the BVH permutation. */
int  rth_scene_permutation(const rth_scene* s, uint32_t* out /* n_tris */);

/* Film::save: divide the accumulated sum by spp and write RLE RGBE (.hdr). */
int  rth_save_hdr(const char* path, int32_t width, int32_t height, const float* rgb_sum, uint32_t spp);
/* Film::tonemap (Imaging.h:233-242) for every pixel: (sum*exposure/(float)spp) clamped at 0,
 * powf(.., 1/2.2f)*255 clamped at 255, truncated to a byte. rgb8 receives width*height*3 bytes. */
int  rth_tonemap(int32_t width, int32_t height, const float* rgb_sum, uint32_t spp, float exposure, uint8_t* rgb8);
/* RayTracer::savePNG (Renderer.h:895-898): tonemapped film written as an 8-bit RGB PNG. */
int  rth_save_png(const char* path, int32_t width, int32_t height, const float* rgb_sum, uint32_t spp);
/* Plain RGBE writer for an already-normalised float RGB image. */
int  rth_write_hdr(const char* path, int32_t width, int32_t height, const float* rgb);
/* Radiance .hdr reader (stbi_loadf semantics, 3 channels). Caller frees with rth_free. */
int  rth_read_hdr(const char* path, int32_t* width, int32_t* height, float** rgb);
/* 8-bit PNG reader (stbi_load semantics). Caller frees with rth_free. */
int  rth_read_png(const char* path, int32_t* width, int32_t* height, int32_t* channels, uint8_t** data);
/* 8-bit texture decode as Texture::load's stbi_load sees it (Imaging.h:50): PNG or JPEG (baseline
 * and progressive) chosen by content; channels = 1 or 3 for JPEG. Free with rth_free. */
int  rth_read_ldr(const char* path, int32_t* width, int32_t* height, int32_t* channels, uint8_t** data);
void rth_free(void* p);

/* C3 synthetic scene: n_tris random triangles, splitmix64 stream from seed,
 * written as .gem + scene.json + albedo .png + constant env.hdr so rth_load_scene loads it. */
int  rth_write_synthetic(const char* dir, uint32_t n_tris, uint64_t seed, int32_t width, int32_t height);
/* The same scene recipe around caller-given triangles (positions: 9 floats per triangle, face normals). */
int  rth_write_mesh_scene(const char* dir, const float* positions, uint32_t n_tris, int32_t width, int32_t height);

#ifdef __cplusplus
}
#endif
#endif /* RTH_H */
