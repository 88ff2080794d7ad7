/* srr -- MI355X-native path tracer: C-ABI drop-in boundary.
 *
 * The reference (truemeat001/Simple-Raytracing-Render) has no FFI: its
 * "operator API" is a C++ class hierarchy that scene builders instantiate with
 * `new` (Raytracing_n.cpp:108-711) and a render driver walks on 8 CPU threads
 * (renderthread, Raytracing_n.cpp:815-879).  This header is that boundary as a
 * flat C ABI: one constructor per reference class (same argument order and
 * meaning), returning integer handles, plus the render entry points that
 * replace renderthread/main.  Plain pointers and sizes only; no C++ or torch
 * types.  Every function returns >= 0 on success and a negative errno-style code
 * on failure (srr_last_error() has the message); nothing calls exit()
 * (the reference's sobol_points does, Raytracing_n.cpp:724-727).
 *
 * Threading: a scene / renderer handle is used by one host thread at a time.
 * The C++ source-compatible headers in include/srr/ are a thin layer over this
 * ABI (see INTEGRATION.md for the ctypes / C++ bindings).
 */
#ifndef SRR_CAPI_H
#define SRR_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRR_OK 0
#define SRR_EINVAL (-22)
#define SRR_ENOMEM (-12)
#define SRR_ENODEV (-19)
#define SRR_ENOTSUP (-95)
#define SRR_EIO (-5)

typedef struct srr_scene srr_scene;
typedef struct srr_renderer srr_renderer;

/* Thread-local message for the last failing call on this thread. */
const char* srr_last_error(void);
/* Library version / build string ("srr 0.1 gfx950 ..."). */
const char* srr_version(void);

/* ------------------------------------------------------------ scene lifetime */
srr_scene* srr_scene_create(void);
void srr_scene_destroy(srr_scene* s);
/* Parse an srr scene description v1 into a new scene. */
int srr_scene_from_text(const char* text, srr_scene** out);
/* Handle of the hitable a parsed description named `obj <text_id>`. */
int srr_scene_text_handle(const srr_scene* s, int text_id);
/* State of the scene-build LCG (the reference's global drand48 seed,
 * mathf.h:12) that the next srr_bvh_node() consumes; default is the
 * post-Perlin state 24561125610955 (perlin.h:94-97). */
int srr_scene_set_lcg(srr_scene* s, uint64_t state);
/* FNV-1a-64 digest of the scene's flattened device tables (no GPU needed): two
 * scenes with equal digests render identically (used to pin scene builders).
 * parts: NULL or SRR_DIGEST_PARTS per-table digests (objects, n_world,
 * transforms, spheres, rects, triangles, meshes, BVH2, BVH4, triangle
 * positions, triangle shading, media, object BVHs, their children, materials,
 * textures, image bytes, Perlin vectors, Perlin permutations, lights, camera). */
#define SRR_DIGEST_PARTS 21
int srr_scene_digest(const srr_scene* s, uint64_t* out, uint64_t* parts);
uint64_t srr_scene_get_lcg(const srr_scene* s);
/* drand48() on the scene LCG (mathf.h:14-19), for builders that draw. */
double srr_scene_drand48(srr_scene* s);

/* ------------------------------------------------------------------ textures
 * texture.h:25-33 constant_texture(vec3) */
int srr_constant_texture(srr_scene* s, float r, float g, float b);
/* texture.h:48-70 image_texture(unsigned char* pixels, int nx, int ny): RGB8,
 * row 0 = top; the bytes are copied (the reference borrows them). */
int srr_image_texture(srr_scene* s, const unsigned char* rgb, int nx, int ny);
/* image_texture(stbi_load(path, &tx, &ty, &tn, 0), tx, ty), the builders' idiom
 * (Raytracing_n.cpp:269-270, :614-616, :631-632): decodes PNG / baseline JPEG /
 * TGA as stb_image v2.19 does (byte-identical, tests/test_imageio.py) and keeps
 * the 3 bytes per texel image_texture addresses. */
int srr_image_texture_file(srr_scene* s, const char* path);
/* Synthetic RGB8 image (stand-in for stbi_load'ed assets; kind 0 sky, 1 wood,
 * 2 checker), identical bytes on every consumer. */
int srr_image_texture_gen(srr_scene* s, int nx, int ny, uint32_t seed, int kind);
/* texture.h:9-23 checker_texture(texture* t0 (even), texture* t1 (odd)) */
int srr_checker_texture(srr_scene* s, int even_tex, int odd_tex);
/* texture.h:35-46 noise_texture(float scale) (Perlin tables of perlin.h:67-97) */
int srr_noise_texture(srr_scene* s, float scale);

/* ----------------------------------------------------------------- materials
 * (material.h); a material handle of -1 is the reference's null material* */
int srr_lambertian(srr_scene* s, int albedo_tex);                       /* :95-114  */
int srr_orennayar(srr_scene* s, int albedo_tex, float sigma_deg);       /* :127-149 */
int srr_beckmann(srr_scene* s, int albedo_tex, float roughx, float roughy); /* :151-199 */
int srr_metal(srr_scene* s, float r, float g, float b, float fuzz);     /* :243-261 */
int srr_dielectric(srr_scene* s, float ref_idx);                        /* :282-339 */
int srr_diffuse_light(srr_scene* s, int emit_tex);                      /* :341-356 */
int srr_isotropic(srr_scene* s, int albedo_tex);                        /* :359-369 */

/* ------------------------------------------------------------------ hitables */
int srr_sphere(srr_scene* s, const float center[3], float radius, int mat);        /* sphere.h:21 */
int srr_moving_sphere(srr_scene* s, const float c0[3], const float c1[3], float t0, float t1, float radius,
                      int mat);                                                     /* moving_sphere.h:8 */
int srr_xy_rect(srr_scene* s, float x0, float x1, float y0, float y1, float k, int mat); /* aarect.h:8 */
int srr_xz_rect(srr_scene* s, float x0, float x1, float z0, float z1, float k, int mat); /* aarect.h:38 */
int srr_yz_rect(srr_scene* s, float y0, float y1, float z0, float z1, float k, int mat); /* aarect.h:69 */
int srr_box(srr_scene* s, const float p0[3], const float p1[3], int mat);          /* box.h:18-29 */
/* triangle.h:13-50: uv (3 x vec3) and normals (3 x vec3) may be NULL; without
 * normals the face normal is used (SURVEY Q5 build definition). */
int srr_triangle(srr_scene* s, const float p[9], int mat, const float* uv9, const float* n9);
int srr_flip_normals(srr_scene* s, int child);                                     /* aarect.h:149-171 */
int srr_translate(srr_scene* s, int child, const float offset[3]);                 /* hitable.h:35-61 */
int srr_rotate_y(srr_scene* s, int child, float angle_deg);                        /* hitable.h:65-132 */
int srr_rotate_x(srr_scene* s, int child, float angle_deg);                        /* hitable.h:135-203 */
int srr_constant_medium(srr_scene* s, int boundary, float density, int tex);       /* constant_medium.h:6 */
int srr_hitable_list(srr_scene* s, const int* children, int n);                    /* hitable_list.h:11 */
/* bvh.h:96-119 bvh_node(hitable** l, int n, float time0, float time1): built
 * eagerly with the reference's random-axis median split, consuming the scene
 * LCG exactly like the reference (one draw per node). */
int srr_bvh_node(srr_scene* s, const int* children, int n, float time0, float time1);
/* Utah teapot (teapot.h:76-166) with `divs` subdivisions: creates 2*32*divs^2
 * triangle handles, first_handle .. first_handle+count-1, returns count. */
int srr_teapot(srr_scene* s, float scale, int divs, int mat, int* first_handle);

/* model.h:27-102 (assimp replaced by srr's PLY / binary-FBX readers): the file's
 * first mesh (model::genhitablemodel returns mesh 0 only) as triangles built like
 * geometry.h:55-77: positions scaled per component, UV channel 0 (v -> 1 - v with
 * flip_uvs), index order reversed with flip_winding, polygons fanned.  Creates
 * count triangle handles first_handle .. first_handle+count-1 and returns count.
 * Files without normals get face normals (SURVEY Q19 build definition). */
int srr_model(srr_scene* s, const char* path, int flip_uvs, int flip_winding, int mat, const float scale[3],
              int* first_handle);
/* The same triangles without a scene: per triangle 9 floats each of positions,
 * uvs (u, v, 0 per corner) and normals (zeros when the file has none; the scene
 * then uses face normals).  Buffers may be NULL to ask for the count.
 * flags_out (may be NULL): bit 0 file has normals, bit 1 file has UVs. */
int srr_mesh_file_triangles(const char* path, int flip_uvs, int flip_winding, const float scale[3], float* pos9,
                            float* uv9, float* nrm9, int* flags_out);

/* camera.h:33-48, 9-argument constructor */
int srr_camera(srr_scene* s, const float lookfrom[3], const float lookat[3], const float vup[3], float vfov,
               float aspect, float aperture, float focus_dist, float t0, float t1);
/* world: the hitable passed as `world` to renderthread (Raytracing_n.cpp:815);
 * lights: `hlist`, must be a hitable_list (cast at Raytracing_n.cpp:75). */
int srr_scene_set_world(srr_scene* s, int obj);
int srr_scene_set_lights(srr_scene* s, int list_obj);

/* ----------------------------------------------------------------- rendering */
typedef struct srr_params {
  int nx, ny;          /* image size (Raytracing_n.cpp:39-40)                  */
  int spp;             /* samples per pixel, ns (:41)                          */
  int max_depth;       /* maxDepth (:42)                                       */
  int tile;            /* tile edge for sharding, e.g. 32                      */
  int shard_index;     /* this renderer renders tiles t (in tile row tr) with  */
  int shard_count;     /*   (t + tr) % shard_count == shard_index */
  int batch_paths;     /* paths in flight per wavefront batch (0 = auto)       */
  uint64_t base_seed;  /* per-path seed salt; 0 = SURVEY §8(d) definition      */
  int flags;           /* SRR_FLAG_*                                           */
  int sample_begin;    /* global index of sample 0: a sample shard renders     */
                       /*   samples [sample_begin, sample_begin + spp)         */
} srr_params;

#define SRR_FLAG_SORT_MATERIALS 1 /* material-sorted shading (perf only)      */
#define SRR_FLAG_KEEP_PATHS 2     /* keep per-path radiance for parity tests   */
#define SRR_FLAG_COUNT_VISITS 4   /* count mesh box / triangle tests (slower)    */
#define SRR_FLAG_WAVEFRONT 8      /* use the wavefront engine (per-bounce kernels) */
                                  /* instead of the path-resident persistent one  */
#define SRR_FLAG_CONTINUE 16      /* progressive rendering: add this render's      */
                                  /* samples to the renderer's per-pixel running   */
                                  /* sums (set sample_begin to the samples already */
                                  /* in them); the mean covers all of them         */
#define SRR_FLAG_SUMS 32          /* srr_render_device writes the per-pixel sample */
                                  /* SUMS (the running sums) instead of the means: */
                                  /* sample-sharded frames reduce these over ranks */

typedef struct srr_stats {
  int64_t world_rays;   /* world->hit calls (the metric's samples)             */
  int64_t paths;        /* camera paths                                        */
  int64_t trace_launches;
  double trace_ms;      /* summed HIP-event time of the trace kernel launches  */
  double shade_ms;
  double total_ms;      /* render wall time on the device stream               */
  int64_t bounces;      /* bounce iterations launched                          */
  int64_t box_tests;    /* SRR_FLAG_COUNT_VISITS: mesh BVH boxes tested        */
  int64_t tri_tests;    /*   triangle tests (a 1-triangle leaf counts 2, as    */
                        /*   the reference tests it twice, bvh.h:104-105)      */
  int64_t stack_overflows; /* rays re-walked on the stackless BVH2             */
  int64_t deep_traversals; /* path engine: mesh traversals whose stack went past */
                           /* its LDS part into the global extension           */
  int64_t mixture_capped;  /* path engine: resampling loops (Raytracing_n.cpp:79-83) */
                           /* stopped by the 100,000-attempt cap   */
  int64_t walks_suspended; /* path engine: mesh walks continued in a later wave-  */
                           /* iteration (SRR_WALK_Q)              */
} srr_stats;

/* Flatten the scene and upload it to HIP device `device`. */
int srr_renderer_create(const srr_scene* s, int device, srr_renderer** out);
void srr_renderer_destroy(srr_renderer* r);
/* One renderer over n_devices GPUs: the replacement for the
 * reference's 8 renderthreads in one process (Raytracing_n.cpp:932-941) at node
 * scale.  The scene is flattened once and uploaded to every device.  srr_render,
 * srr_render_device, srr_render_device_async and srr_render_wait on the handle
 * render the WHOLE frame (shard_index / shard_count must be 0 / 0 or 1): tiles of
 * edge p->tile (<= 0: 32) dealt round-robin over the devices, each tile row
 * rotated by one (srr_shard_pixels with shard_count = n_devices), all devices at
 * once, then ONE frame-end gather of the packed shard slabs to device_ids[0] over
 * RCCL (ncclCommInitAll communicator, ncclSend / ncclRecv in one group) and a
 * scatter into the image there: d_mean is a device_ids[0] pointer of nx*ny*3
 * floats, bitwise the one-device frame.  srr_render / srr_render_device return
 * after the gather; srr_render_device_async enqueues the gather on the GPU behind
 * the shards' frames (and behind the caller's legacy-stream work on device_ids[0])
 * and returns at once -- the host waits only in srr_render_wait.
 * device_ids may repeat a device (a rehearsal on one GPU): the gather is then
 * device copies, as with SRR_MULTI_TRANSPORT=copy.  No KEEP_PATHS / CONTINUE
 * (SRR_EINVAL); srr_accum_* and srr_copy_paths are single-device. */
int srr_renderer_create_multi(const srr_scene* s, int n_devices, const int* device_ids, srr_renderer** out);
/* Devices a renderer renders on (1 for srr_renderer_create), ids into
 * device_ids[0 .. cap) (may be NULL). */
int srr_renderer_devices(const srr_renderer* r, int* device_ids, int cap);
/* The frame-end transport of a renderer: "rccl", "copy", or "none" (one device). */
const char* srr_renderer_transport(const srr_renderer* r);
/* The multi-device frame's bookkeeping, host only (no GPU): shard k's pixels are
 * srr_shard_pixels({.., shard_index k, shard_count n_devices}); the gather packs
 * the shards' slabs in shard order, so packed entry i is image pixel
 * gather_index[i] (nx*ny entries, may be NULL) and shard k's slab starts at
 * shard_offsets[k] (n_devices + 1 entries, may be NULL).  Returns nx*ny. */
int64_t srr_multi_plan(const srr_params* p, int n_devices, int32_t* gather_index, int64_t* shard_offsets);
/* Number of pixels this shard renders, and their PPM-order indices (row 0 =
 * top, Raytracing_n.cpp:873-876) into pixel_index[] (may be NULL). */
int64_t srr_shard_pixels(const srr_params* p, int32_t* pixel_index);
/* Render this shard.  d_mean: DEVICE pointer, n_shard_pixels*3 floats -- the
 * per-pixel mean of de_nan'd samples before the sqrt (Raytracing_n.cpp:841-848),
 * in srr_shard_pixels() order.  Inputs are resident on the device; the call
 * returns after the device work finished. */
int srr_render_device(srr_renderer* r, const srr_params* p, float* d_mean, srr_stats* stats);
/* Frame pipelining (no reference counterpart: the reference renders one frame
 * per run).  Enqueue the same frame as srr_render_device and return at once with
 * a ticket; the renderer keeps two frames in flight on two streams, so a frame's
 * persistent blocks start on the CUs the previous frame's last paths free.  Fresh
 * frames of the path engine only (no CONTINUE, KEEP_PATHS, COUNT_VISITS,
 * WAVEFRONT: SRR_EINVAL).  d_mean must not be read, and must not be the target
 * of another frame in flight, before srr_render_wait(ticket) returns; enqueueing
 * a third frame first finishes the oldest (its stats stay for its wait).
 * Device memory: each frame in flight holds its own sample window (all shard
 * pixels x the window's samples x 12 B, at most SRR_WINDOW_MB, default 16 GiB),
 * bounce records (16 B x max_depth per persistent lane) and sums; the
 * synchronous slot keeps its own window too, so alternating the two modes
 * reallocates nothing (the other mode's windows are given back only when an
 * allocation would run the device out of memory).  Per renderer the windows are
 * thus at most 3 x SRR_WINDOW_MB; the peers of a multi-device renderer that share
 * a device (device_ids repeating it) split SRR_WINDOW_MB between them, so a
 * device holds at most 3 x SRR_WINDOW_MB of windows either way. */
int srr_render_device_async(srr_renderer* r, const srr_params* p, float* d_mean, int64_t* ticket);
/* Wait for an async frame and return its stats (each ticket once). */
int srr_render_wait(srr_renderer* r, int64_t ticket, srr_stats* stats);
/* Host convenience (the CRender::Run of Render.h:16-51): the shard's pixels
 * (the whole image when shard_count <= 1) as mean radiance (npix*3, may be NULL)
 * and 8-bit tone-mapped rgb8 (npix*3, Raytracing_n.cpp:850-867, may be NULL). */
int srr_render(srr_renderer* r, const srr_params* p, float* mean, unsigned char* rgb8, srr_stats* stats);
/* Progressive rendering with resume: the renderer's per-pixel running sums
 * (3 floats per shard pixel, in srr_shard_pixels order) and the samples per pixel
 * they hold.  get: sums may be NULL to query npix / samples.  set: restores a saved
 * state, after which renders with SRR_FLAG_CONTINUE and sample_begin = samples
 * continue it (bitwise the image of one render of all the samples). */
int srr_accum_get(srr_renderer* r, float* sums, int64_t* npix, int64_t* samples);
int srr_accum_set(srr_renderer* r, const float* sums, int64_t npix, int64_t samples);
/* After a render with SRR_FLAG_KEEP_PATHS: per-path raw radiance (before
 * de_nan) and world-ray counts, [n_shard_pixels][spp]. */
int srr_copy_paths(srr_renderer* r, float* radiance, unsigned char* rays);
/* ---- MERL measured isotropic BRDF tables (brdf.h).  The reference reads a
 * table (brdf::read_brdf, brdf.h:156-185) and looks values up by half/difference
 * angles (brdf::lookup_brdf_val, :190-214); its only user, brdfmaterial
 * (material.h:201-241), never sets a pdf and is never placed in a scene
 * (SURVEY Q23), so the lookup is exposed on its own. */
typedef struct srr_merl srr_merl;
/* brdf::read_brdf: int32 dims[3], then 3 * dims[0]*dims[1]*dims[2] doubles
 * (channel-major); the product must be 90*90*180 (else SRR_EINVAL, the
 * reference's "Dimensions don't match").  Uploads the table to HIP device `device`. */
int srr_merl_load(const char* path, int device, srr_merl** out);
/* The same from memory: n_doubles must be 3*90*90*180. */
int srr_merl_create(const double* table, int64_t n_doubles, int device, srr_merl** out);
void srr_merl_destroy(srr_merl* m);
/* brdf::lookup_brdf_val for n queries on the device.  angles: 4n doubles
 * (theta_in, fi_in, theta_out, fi_out); rgb: 3n doubles out (RED/GREEN/BLUE_SCALE
 * applied, brdf.h:11-13); cell: n table indices out (may be NULL).  Host buffers.
 * (The reference's "Below horizon." stderr message is not printed.) */
int srr_merl_lookup(srr_merl* m, int64_t n, const double* angles, double* rgb, int32_t* cell);

/* Tone map (Raytracing_n.cpp:850-867): 8-bit = clamp(int(255.99*sqrt(m))). */
int srr_tonemap(const float* mean, int64_t n_pixels, unsigned char* rgb8);
/* Write an ASCII P3 PPM (Raytracing_n.cpp:886, 873-876). */
int srr_write_ppm(const char* path, int nx, int ny, const unsigned char* rgb8);

/* PNG (8-bit RGB) of the tone-mapped image -- the output option next to PPM. */
int srr_write_png(const char* path, int nx, int ny, const unsigned char* rgb8);
/* stbi_load(path, x, y, comp, req_comp) (stb_image.h v2.19, used throughout
 * Raytracing_n.cpp): PNG, baseline JPEG, TGA.  *comp = the file's channels;
 * returns the channels in *out (req_comp, or *comp when req_comp is 0) or a
 * negative code.  Free *out with srr_image_free. */
int srr_image_load(const char* path, int req_comp, int* x, int* y, int* comp, unsigned char** out);
void srr_image_free(unsigned char* pixels);

/* Test infrastructure: run the device (HIP) implementation of one reference
 * function on KAT records laid out as oracle/ref/kat.inc writes them (inputs
 * first, outputs overwritten in place): "erf", "beckmann11", "beckmann_dist",
 * "beckmann_pdf", "cosine_pdf", "orennayar_pdf", "dielectric", "metal",
 * "triangle", "aabb"; and "sqrt" (records x, sqrtf(x)).  Needs a GPU. */
int srr_device_kat(const char* name, int n, int width, float* records);

/* Sobol (0,2)-points of Raytracing_n.cpp:721-812, out[n][2]. */
int srr_sobol_points(int n, double* out);

/* Host-side inspection (no GPU needed) -------------------------------------
 * Teapot triangles (p0 p1 p2, 9 floats each) as srr_teapot would create them;
 * returns the triangle count (out may be NULL to query it). */
int srr_teapot_vertices(float scale, int divs, float* out);
/* Topology of the bvh_node `obj` in preorder, one line per node: "N" for an
 * interior node, "L a b" for a leaf over children a, b (indices into the
 * children array given to srr_bvh_node; a == b for a one-child leaf), after a
 * first line "box minx miny minz maxx maxy maxz".  Returns bytes needed. */
int64_t srr_bvh_topology(const srr_scene* s, int obj, char* buf, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SRR_CAPI_H */
