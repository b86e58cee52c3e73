/*
 * rtx.h — C ABI of librtx.so, the MI355X-native render path of the python-raytracer
 * drop-in (SpacewaIker/python-raytracer @ 2025-02-14).
 *
 * The reference is pure Python, so it has no FFI of its own. Each entry point below
 * replaces one reference interface on the hot path (cited file:line) and is what a
 * ctypes binding of that interface binds:
 *
 *   rtx_scene_create   <- scene_parser.load_scene's object construction
 *                         (provided/scene_parser.py:104-294, geometry ctors in
 *                         provided/geometry/simple_geometry.py:15-18,87-103,180-186,
 *                         provided/geometry/mesh.py:17-70 and
 *                         provided/geometry/hierarchy.py:12-40, textures
 *                         scene_parser.py:222-247): scene objects -> HBM
 *   rtx_camera_set     <- ViewportCamera + the per-frame setup of Scene.render
 *                         (provided/helperclasses.py:69-108, provided/scene.py:36-45)
 *   rtx_render         <- Scene.render's pixel/sample loops + cast_ray + shading
 *                         (provided/scene.py:47-79, :81-116, :140-187, :189-209)
 *   rtx_intersect      <- the Geometry.intersect plugin ABI + closest-hit selection
 *                         (provided/geometry/__init__.py:47-48, provided/scene.py:86-94)
 *   rtx_occluded       <- the Geometry.shadow_intersect plugin ABI + any-hit loop
 *                         (provided/geometry/__init__.py:50-51, provided/scene.py:160-164)
 *   rtx_fb_to_rgb8     <- main.py's rot90 + truncating uint8 conversion
 *                         (provided/main.py:31-33; rot90 is the fb's row order)
 *
 * Conventions
 *   - Every function returns RTX_OK (0) or a negative rtx_status; no C++ exception
 *     crosses the ABI. rtx_last_error() returns a thread-local message for the last
 *     failure on the calling thread.
 *   - Host pointers are read during the call only. Pointers named *_dev are device
 *     (HBM) pointers owned by the caller; the library never frees them.
 *   - rtx_render / rtx_intersect / rtx_occluded / rtx_fb_to_rgb8 are asynchronous on
 *     the given HIP stream (hipStream_t passed as void*; NULL = the default stream).
 *     Scene and camera uploads are synchronous: rtx_camera_set waits for the device to
 *     go idle and copies its tables with a kernel on the null stream, so it must not be
 *     called while any stream is capturing a graph.
 *   - Renders of ONE scene must be stream-ordered (one stream, or events between them):
 *     the hierarchy/texture scenes' split passes keep per-scene scratch (record arrays,
 *     counters, the redo list) that every render of the scene reuses. A render may be
 *     captured into a HIP graph once the scene has rendered eagerly at that size (the
 *     scratch is allocated then); the scene's own buffers live until rtx_scene_destroy.
 *     A captured graph is INVALID after rtx_camera_set: the camera's tables may move and
 *     the kernel it launches was specialized on the old camera (and may be unloaded), so
 *     record it again after every camera upload.
 *   - One device per scene (the current HIP device at rtx_scene_create).
 *   - Numbers carry the reference's types: PyGLM vec3 values are float (fp32), Python
 *     scalars are double (fp64).
 */
#ifndef RTX_H
#define RTX_H

#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 5

typedef enum rtx_status {
    RTX_OK = 0,
    RTX_ERR_INVALID = -1,     /* bad argument / inconsistent description */
    RTX_ERR_HIP = -2,         /* HIP runtime error (message in rtx_last_error) */
    RTX_ERR_UNSUPPORTED = -3, /* feature not built (e.g. textures, hierarchy nodes) */
    RTX_ERR_STATE = -4        /* e.g. rtx_render before rtx_camera_set */
} rtx_status;

typedef enum rtx_object_type { RTX_SPHERE = 0, RTX_PLANE = 1, RTX_BOX = 2, RTX_MESH = 3, RTX_NODE = 4 } rtx_object_type;
typedef enum rtx_hierarchy_type {
    RTX_UNION = 0, RTX_INTERSECTION = 1, RTX_DIFFERENCE = 2, RTX_HIER_OTHER = 3  /* other: no hits */
} rtx_hierarchy_type;
typedef enum rtx_material_type { RTX_MAT_DIFFUSE = 0, RTX_MAT_MIRROR = 1, RTX_MAT_REFRACTIVE = 2 } rtx_material_type;
typedef enum rtx_light_type { RTX_LIGHT_POINT = 0, RTX_LIGHT_DIRECTIONAL = 1 } rtx_light_type;
typedef enum rtx_bv_type { RTX_BV_AABB = 0, RTX_BV_SPHERE = 1 } rtx_bv_type;
typedef enum rtx_jitter_mode { RTX_JITTER_OFF = 0, RTX_JITTER_PHILOX = 1, RTX_JITTER_REPLAY = 2 } rtx_jitter_mode;

/* One geometry record. Top-level objects (parent == -1) are in scene (JSON) order, which
 * is the closest-hit tie break (min() keeps the first minimum, provided/scene.py:94).
 * Hierarchy nodes (RTX_NODE, provided/geometry/hierarchy.py) are followed by their
 * subtree in preorder: every record after a node whose parent is that node is one of
 * its children, in child order. Child records carry what the parser gives them:
 * materials after Hierarchy.set_fallback_material (hierarchy.py:21-28), speeds after
 * traverse_children's `speed + child speed` (scene_parser.py:268-271). */
typedef struct rtx_object {
    int32_t type;          /* rtx_object_type */
    int32_t n_mats;        /* associated materials (Plane: 1 = plain, >=2 = checker) */
    int32_t mat[2];        /* material indices; mat[0] for sphere / box / mesh */
    int32_t has_speed;     /* 0 = speed None; else position + speed * time */
    float speed[3];
    float a[3];            /* sphere centre | plane point | box minpos | (mesh unused) */
    float b[3];            /* plane normal  | box maxpos */
    double radius;         /* sphere radius (Python float) */
    int32_t tri_begin;     /* mesh: first triangle in rtx_scene_desc.triangles */
    int32_t tri_count;     /* mesh: number of triangles (faces in OBJ order) */
    int32_t bv_type;       /* mesh: rtx_bv_type chosen by Mesh.__init__ (mesh.py:44-51) */
    int32_t flat;          /* mesh: flat_shaded */
    float bv_a[3];         /* mesh BV: AABB min | sphere centre */
    float bv_b[3];         /* mesh BV: AABB max */
    double bv_radius;      /* mesh BV: sphere radius (Python float) */
    int32_t parent;        /* -1: top-level; else index of the enclosing RTX_NODE record */
    int32_t hierarchy_type;/* node: rtx_hierarchy_type */
    float trs[9];          /* node: position, rotation (degrees), scale (Hierarchy.make_matrices) */
    int32_t texture;       /* plane / box: index into rtx_scene_desc.textures, -1 = none */
    double texture_scale;  /* plane: texture_scale (scene_parser.py:226, default 1.0) */
} rtx_object;

/* A texture as Image.getpixel sees it (scene_parser.py:224, simple_geometry.py:168):
 * rgb[3 * (j * width + i) + c] = getpixel((i, j))[c]. */
typedef struct rtx_texture {
    int32_t width, height;
    const uint8_t* rgb;
} rtx_texture;

/* One mesh face after Mesh.__init__'s (v + translate) * scale transform (mesh.py:24),
 * with the per-vertex smooth normals of _compute_normals (mesh.py:53-70; ignored
 * when the mesh is flat shaded). */
typedef struct rtx_triangle {
    float v0[3], v1[3], v2[3];
    float n0[3], n1[3], n2[3];
} rtx_triangle;

typedef struct rtx_material {
    float diffuse[3];
    float specular[3];
    double hardness;       /* Python number; `x ** hardness` in fp64 */
    int32_t type;          /* rtx_material_type */
    double tint;
    double refr_index;
} rtx_material;

typedef struct rtx_light {
    int32_t type;          /* rtx_light_type */
    float colour[3];
    float vector[3];       /* position (point) | direction (directional) */
    double power;          /* directional lights: 1.0 (scene_parser.py:116-118) */
} rtx_light;

typedef struct rtx_scene_desc {
    int32_t n_objects;
    const rtx_object* objects;
    int32_t n_materials;
    const rtx_material* materials;
    int32_t n_lights;
    const rtx_light* lights;
    int32_t n_triangles;
    const rtx_triangle* triangles;
    float ambient[3];
    int32_t n_textures;
    const rtx_texture* textures;
} rtx_scene_desc;

/* Per-frame camera state. Tables are the reference's scalar sequences, evaluated on the
 * host exactly as provided/scene.py computes them. */
typedef struct rtx_camera_desc {
    int32_t width, height;   /* full image size */
    int32_t col0, ncols;     /* rendered column strip (np.array_split range of Scene.render) */
    const float* xs;         /* [ncols] fp32 of the fp64 x running sum (scene.py:42,77) */
    const float* ys;         /* [height] fp32 of the fp64 y running sum, bottom row first (scene.py:48,75) */
    float position[3];
    float u[3], v[3], w[3];
    double d;                /* ViewportCamera.d (1.0) */
    double focal_length;
    int32_t n_dof, n_aa;
    const float* dof_origins;/* [n_dof][3] _sunflower_spread(dof, position, aperture) */
    const float* aa_origins; /* [n_dof][n_aa][3] _sunflower_spread(aa, dof_origin, 2(dx+dy)) */
    int32_t n_times;
    const double* times;     /* [n_times] ViewportCamera.motion_times */
    int32_t jitter;          /* rtx_jitter_mode */
    double jitter_scale;     /* 0.1 * (dx + dy) (scene.py:64) */
    uint64_t seed;           /* RTX_JITTER_PHILOX key */
    const float* noise;      /* RTX_JITTER_REPLAY: host [ncols][height][n_dof][n_aa][3] values of
                                np.random.rand() in the reference's call order (i, j, dof, aa) */
} rtx_camera_desc;

/* Device counters written by rtx_render when counters_dev != NULL (uint64[RTX_COUNTERS]). */
#define RTX_COUNTERS 16
#define RTX_CNT_CAST0 0      /* [0..9]: cast_ray calls that intersect, by recursion depth */
#define RTX_CNT_SHADOW 10    /* shadow rays */
#define RTX_CNT_SHADE 11     /* _compute_regular_lighting calls */
#define RTX_CNT_TRI 12       /* ray-triangle tests */

typedef struct rtx_scene rtx_scene;

int rtx_abi_version(void);
const char* rtx_last_error(void);

int rtx_scene_create(const rtx_scene_desc* desc, rtx_scene** out);
int rtx_scene_destroy(rtx_scene* scene);
int rtx_camera_set(rtx_scene* scene, const rtx_camera_desc* cam);

/* Renders image rows [row0, row0 + nrows) (row 0 = top of the PNG) of the camera's
 * column strip into fb_dev: float32 [nrows][ncols][3], i.e. the reference image
 * rotated by main.py's rot90. */
int rtx_render(rtx_scene* scene, int32_t row0, int32_t nrows, float* fb_dev,
               uint64_t* counters_dev, void* hip_stream);

/* Multi-GPU load balance (no reference counterpart: the reference splits columns across
 * processes, provided/scene.py:36-37 + render.nu): renders the 8-row groups phase,
 * phase + stride, phase + 2 stride, ... of the image (row 0 = top), packed in order into
 * fb_dev: float32 [rtx_group_rows(height, phase, stride)][ncols][3]. Rank r of N calls
 * it with (r, N), so every rank gets rows from the whole frame (sky and ground alike).
 * Pixel values equal rtx_render's for the same rows. */
int rtx_render_groups(rtx_scene* scene, int32_t phase, int32_t stride, float* fb_dev,
                      uint64_t* counters_dev, void* hip_stream);

/* rtx_render / rtx_render_groups with main.py's PNG conversion fused into the render
 * (provided/main.py:31-33): out_dev receives uint8 [rows][ncols][3] = (v * 255.0) truncated
 * of the fp32 values rtx_render would write — identical bytes to rtx_render followed by
 * rtx_fb_to_rgb8, with 4x fewer bytes stored (and gathered, across ranks). */
int rtx_render_rgb8(rtx_scene* scene, int32_t row0, int32_t nrows, uint8_t* out_dev,
                    uint64_t* counters_dev, void* hip_stream);
int rtx_render_groups_rgb8(rtx_scene* scene, int32_t phase, int32_t stride, uint8_t* out_dev,
                           uint64_t* counters_dev, void* hip_stream);

/* Frames of one scene state in ONE launch (no reference counterpart: a launch-count
 * optimisation of the multi-GPU frame loop, rtx.distributed.FrameExchange): nframes
 * copies of rtx_render (rgb8 = 0: fp32) / rtx_render_rgb8 (rgb8 != 0) of rows
 * [row0, row0 + nrows), frame f at out_dev + f * frame_stride_bytes (>= one frame's
 * bytes; a multiple of 4 for fp32). gridDim.y = nframes fills the GPU that one
 * 1/N-of-a-frame launch per rank leaves partly idle at N = 8. 1 <= nframes <= 65535. */
int rtx_render_frames(rtx_scene* scene, int32_t row0, int32_t nrows, void* out_dev, int32_t rgb8, int32_t nframes,
                      int64_t frame_stride_bytes, uint64_t* counters_dev, void* hip_stream);
/* The same for rtx_render_groups / rtx_render_groups_rgb8 (interleaved 8-row groups). */
int rtx_render_groups_frames(rtx_scene* scene, int32_t phase, int32_t stride, void* out_dev, int32_t rgb8,
                             int32_t nframes, int64_t frame_stride_bytes, uint64_t* counters_dev, void* hip_stream);

/* Rows rtx_render_groups writes for an image of `height` rows (-1: bad arguments). */
int32_t rtx_group_rows(int32_t height, int32_t phase, int32_t stride);

/* Closest hit of n rays (SoA device arrays ray_o_dev/ray_d_dev = [3][n] fp32) at one
 * motion time. Outputs: t (fp64, +inf on miss), object index (-1), material index (-1),
 * normal [3][n], position [3][n]. Any output pointer may be NULL. */
int rtx_intersect(rtx_scene* scene, int64_t n, const float* ray_o_dev, const float* ray_d_dev,
                  double time, double* t_dev, int32_t* obj_dev, int32_t* mat_dev,
                  float* normal_dev, float* position_dev, void* hip_stream);

/* Any-hit shadow test of n rays against every object with per-ray t_max (fp64). */
int rtx_occluded(rtx_scene* scene, int64_t n, const float* ray_o_dev, const float* ray_d_dev,
                 const double* t_max_dev, double time, uint8_t* occluded_dev, void* hip_stream);

/* out_dev[i] = (uint8)(fb_dev[i] * 255.0) in fp64 with truncation (main.py:33). */
int rtx_fb_to_rgb8(const float* fb_dev, uint8_t* out_dev, int64_t n_values, void* hip_stream);

/* Observability (no reference counterpart): the name of the kernel the last
 * rtx_render / rtx_render_groups call on this scene launched — "rtx_jit_render_<flags>"
 * for a scene-specialized (hiprtc) kernel, "k_render_<flags>" / "k_render_ext_<flags>"
 * for the precompiled generic ones; "" before the first render. Valid until the next
 * render call on the scene or rtx_scene_destroy. */
const char* rtx_last_kernel(const rtx_scene* scene);

/* Observability (no reference counterpart): the number of scene-specialized kernel
 * modules loaded in this process. Kernels whose source carries one scene's record values
 * are unloaded once no scene holds them and more than jit_idle_baked (option, default 8)
 * such idle modules exist, so the count stays bounded as scenes come and go. */
int32_t rtx_jit_modules(void);

/* Library options (no reference counterpart; INTEGRATION.md "Options"): process-wide
 * switches of the culling structures, the split hierarchy passes, the scene-specialized
 * kernels and their caches, by name ("split", "bins", "jit", ...). Each starts from
 * $RTX_<NAME> when that is set in the environment, else from its default; set them before
 * rendering (they are read per render / per camera upload, not synchronised with renders
 * on other threads). Values are text: a number, or a string for "jit_cache" / "jit_flags".
 * RTX_ERR_INVALID for an unknown name or a malformed number. */
int rtx_set_option(const char* name, const char* value);
/* The option's current value as text into value[cap] (RTX_ERR_INVALID if it does not fit). */
int rtx_get_option(const char* name, char* value, int32_t cap);
/* Name of option i (0, 1, ...; NULL past the last). */
const char* rtx_option_name(int32_t i);

/* Scene-specialized kernels compiled on a host thread (option jit_async, default 1; no
 * reference counterpart): a scene's first renders launch the precompiled generic kernel,
 * which renders the same bytes, while hiprtc compiles the specialized one; a later render
 * that finds the compile done switches to it. rtx_jit_wait picks up the scene's finished
 * compiles -- block != 0: waits for all of them first -- and returns how many are still
 * compiling (0 once every kernel the scene's camera has rendered with is resolved). */
int32_t rtx_jit_wait(rtx_scene* scene, int32_t block);

/* Multi-GPU frame loop (no reference counterpart; the reference's strip renders and glue,
 * render.nu:10-15 + provided/glue.py:17-27, as one HIP graph per frame): launches the
 * instantiated graph graph_exec (a hipGraphExec_t, e.g. one rank's render + RCCL gather of
 * a frame captured by rtx.distributed.FrameGraph) n times in order on hip_stream, from C,
 * so a frame costs one hipGraphLaunch of host time. Asynchronous; RTX_ERR_INVALID for a
 * null graph or n < 0. */
int rtx_graph_launch(void* graph_exec, int32_t n, void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* RTX_H */
