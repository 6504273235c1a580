// om_layout.h — frozen-world layout in HBM (host builder <-> HIP kernels).
//
// The reference keeps one typed Vec per primitive type (hits.rs:34-69, order
// hits.rs:370-371).  The frozen device world keeps that order but splits every
// primitive into a hot "test" record (what a miss needs: 64 B, read by every
// lane of a wave at the same address -> scalar loads) and a cold "hit" record
// (what the winner needs to build its HitRecord).  Global primitive index gi
// follows the type order; obj_id = gi + 1 (0 = sky).
#pragma once
#include <stdint.h>

#define OM_ALIGN16 __attribute__((aligned(16)))

// Affine primitive (Sphere traced.rs:13-19, Cube traced.rs:229-235).
// w2l rows 0..2 (row-major 3x4); dz[i] = w2l[i][3] * 0.0f — the w-term of
// Mat4x4::dot_v3 (mat4x4.rs:54-57) kept so signed zeros match bit for bit.
struct OM_ALIGN16 OmAffineTest {
    float w2l[12];
    float dz[3];
    float pad;
};
struct OM_ALIGN16 OmAffineHit {
    float l2w[12];
    float lz[3];  // l2w[i][3] * 0.0f
    float pad;
};
// Conservative world-space bounding sphere of an affine primitive: center, and
// the inflated radius squared.  Used only to skip exact tests
// that would return None.
struct OM_ALIGN16 OmBound {
    float c[3];
    float r;     // inflated radius
};

// Barycentric<BT> (traced.rs:118-131) — only what hit_aux reads.
struct OM_ALIGN16 OmBary {
    float origin[3];
    float u_length;
    float uxv[3];
    float v_length;
    float base_inv[9];
    float vx, vy;     // v_in_base.x, v_in_base.z (calc_barycentric traced.rs:156-167)
    float pad;
};
// InfinitePlane (traced.rs:77-82)
struct OM_ALIGN16 OmPlane {
    float center[3];
    float pad0;
    float normal[3];
    float pad1;
};
// MarchedSphere (marched.rs:50-54), MarchedBox (marched.rs:79-83)
struct OM_ALIGN16 OmMSphere {
    float center[3];
    float radius;
};
struct OM_ALIGN16 OmMBox {
    float center[3];
    float pad0;
    float sizes[3];
    float br;         // march cull: upper bound of |sizes| (the box lies within |p - center| <= |sizes|)
};
// MarchedTorus (marched.rs:105-113)
struct OM_ALIGN16 OmMTorus {
    float l2w_tr[16];
    float w2l_tr[16];
    float l2w_s[4];
    float w2l_s[4];
    float sizes[3];
    float min_scale;  // l2w_s.xyz().min_val() (marched.rs:148-150), precomputed
    // conservative cull of the SDF evaluation (march): |sdf(p)| >= |p - bc| / bk - br,
    // all with margins, so a step skips the torus when that bound already exceeds the
    // running minimum
    float bc[3];      // world centre: translation of l2w_tr scaled by l2w_s
    float bk;         // upper bound of (max scale) / min_scale-margined factor (see om_world.cpp)
    float br;         // upper bound of (R + r) / min-w2l_s factor
    float pad_b[3];
};
// A user marched object (`HittableList += Arc<dyn Marched>`, hits.rs:96-100; om_world_add_marched_sdf):
// MarchedTorus's transform fields (same names, so the torus's to_local / normal code serves both)
// and its local_sdf as a postfix program ops[op_first .. op_first + op_count) (OmSdfOp).
struct OM_ALIGN16 OmMSdf {
    float l2w_tr[16];
    float w2l_tr[16];
    float l2w_s[4];
    float w2l_s[4];
    float min_scale;  // l2w_s.xyz().min_val(): to_world_f (marched.rs:148-150)
    uint32_t op_first, op_count, pad;
};
struct OM_ALIGN16 OmSdfOp {
    uint32_t op;      // OM_SDF_* (ottomarcher.h)
    float a[7];
};

// Material (materials.rs:18-24), padded to 32 B.
struct OM_ALIGN16 OmMaterial {
    float albedo[3];
    float fuzz;
    float ior;
    int32_t type;
    float pad[2];
};

// BVH node (binary, 32 B).  Internal: left/right children; leaf: [first, first+count)
// into the prim index list.  Boxes are conservative (inflated).
struct OM_ALIGN16 OmBvhNode {
    float lo[3];
    int32_t left;     // >=0 internal: index of left child; <0 leaf: -(first+1)
    float hi[3];
    int32_t right;    // internal: index of right child; leaf: count
};

// Stackless BVH node (32 B), depth-first order: on a box hit go to idx+1 (internal)
// or test the leaf's records then go to `skip`; on a miss go to `skip`.
// leaf = (first_record << 8) | count, or 0xFFFFFFFF for an internal node.
struct OM_ALIGN16 OmSkipNode {
    float lo[3];
    uint32_t skip;
    float hi[3];
    uint32_t leaf;
};

// 4-wide BVH node (112 B), collapsed from the BVH2: up to four child boxes (SoA per
// axis) and 16-bit child codes (node index | OM_LEAF + leaf index | OM_EMPTY).  Same
// leaf table and records as the BVH2.
#define OM_EMPTY 0xFFFFu
struct OM_ALIGN16 OmBvh4Node {
    float lox[4], loy[4], loz[4], hix[4], hiy[4], hiz[4];
    uint16_t child[4];
    uint32_t pad[2];
};

// The 4-wide node with half-precision child boxes (64 B, one cache line; trees read through L2):
// planes rounded outward like OmBvh2NodeH, b = lox[4] loy[4] loz[4] hix[4] hiy[4] hiz[4].  Emitted
// breadth-first, so an LDS prefix holds the top levels (om_wavefront.hip, OM_WF_HYB4_BYTES).
struct OM_ALIGN16 OmBvh4NodeH {
    uint16_t b[24];
    uint16_t child[4];
    uint32_t pad[2];
};

// Prim tested outside the BVH2 tree (always2), with a conservative box tested first:
// inflated for triangles/parallelograms, infinite for planes and huge bounds.
struct OM_ALIGN16 OmAlwaysRec {
    float lo[3];
    uint32_t gi;
    float hi[3];
    uint32_t pad;     // OM_ALWAYS_DIAG_SPHERE: a sphere whose world-to-local block is diagonal
};
#define OM_ALWAYS_DIAG_SPHERE 1u

// Compressed binary BVH node (64 B): both child boxes live in the parent, so one
// node read yields both slab tests.  child = 16-bit code: node index, or
// OM_LEAF | leaf index; b2leaves[leaf] = (first_record << 8) | count (records =
// srecs, leaf order), or, when the records fit (om_bvh.cpp), the direct code
// OM_LEAF | first << 4 | count.  The traversal stack holds these 16-bit codes.
#define OM_LEAF 0x8000u
struct OM_ALIGN16 OmBvh2Node {
    float lo0[3];
    uint32_t c0;
    float hi0[3];
    uint32_t pad0;
    float lo1[3];
    uint32_t c1;
    float hi1[3];
    uint32_t pad1;
};
#define OM_B2_LO(n, k, i) ((k) == 0 ? (n).lo0[i] : (n).lo1[i])
#define OM_B2_HI(n, k, i) ((k) == 0 ? (n).hi0[i] : (n).hi1[i])
// The compressed form of the same node (32 B, r04; trees too big for LDS): the child boxes as IEEE half-precision bits,
// each plane rounded OUTWARD (lo down, hi up) from the f32 box, so a decoded box contains the
// f32 one and the culling stays conservative (boxes only decide which exact tests run).  A visit
// reads two 16-B words instead of four, and the slab test's fma takes the halves directly
// (v_fma_mix_f32: no extra VALU).  b: child 0 lo xyz, hi xyz; child 1 lo xyz, hi xyz.
struct OM_ALIGN16 OmBvh2NodeH {
    uint16_t b[12];
    uint16_t c0, c1;
    uint32_t pad;
};
// f32 BVH2 nodes + leaf table of at most this many bytes are staged whole in LDS per workgroup;
// a bigger tree is read through L2 (half nodes, an LDS prefix) and built with smaller leaves
constexpr uint32_t kB2LdsBudget = 40u * 1024u;

// Device view of a frozen world (passed by value as a kernel argument).
struct OmSceneDev {
    const OmAffineTest* sph_test; const OmAffineHit* sph_hit; const OmBound* sph_bound;
    const OmAffineTest* cube_test; const OmAffineHit* cube_hit; const OmBound* cube_bound;
    const OmBary* tri; const OmPlane* plane; const OmBary* para;
    const OmMSphere* msph; const OmMBox* mbox; const OmMTorus* mtor;
    const OmMSdf* msdf; const OmSdfOp* msdf_ops;   // user marched objects (after the tori in gi order)
    const OmMaterial* mats;       // by global index gi
    const uint64_t* bloom;        // by obj_id (gi + 1); bloom[0] = 0
    const OmBvhNode* bvh;         // over bounded traced prims (spheres, cubes, tris, paras)
    const uint32_t* bvh_prims;    // leaf -> global index gi
    uint32_t n_sph, n_cube, n_tri, n_plane, n_para, n_msph, n_mbox, n_mtor, n_msdf;
    uint32_t n_bvh_nodes;
    uint32_t n_always;            // number of unbounded/huge prims tested outside the BVH
    const uint32_t* always;       // their global indices (ascending)
    // type offsets of the global index space
    uint32_t off_cube, off_tri, off_plane, off_para, off_msph, off_mbox, off_mtor, off_msdf, n_total;
    // stackless BVH over the affine primitives (records carry gi | cube<<31 in `pad`)
    const OmSkipNode* snodes; const OmAffineTest* srecs; const uint32_t* always2;
    uint32_t n_snodes, n_srecs, n_always2;
    uint32_t lds_bytes;           // dynamic LDS the staged kernel needs (0 = scene too big: global path)
    // compressed BVH2 over the same leaves/records as the stackless BVH
    const OmBvh2Node* b2nodes;    // f32 nodes (trees staged whole in LDS; the megakernel)
    const OmBvh2NodeH* b2h;       // the same nodes with half-precision boxes (trees read through L2)
    const uint32_t* b2leaves;
    const OmAlwaysRec* always2_rec;  // always2 with boxes (BVH2 traversal)
    uint32_t n_b2nodes, n_b2leaves;
    uint32_t b2_lds_bytes;        // node bytes when they fit the LDS budget, else 0 (global nodes)
    uint32_t b2_stack;            // lane-stack entries the tree needs (its internal depth, <= 24)
    uint32_t b2_direct;           // leaf codes are OM_LEAF | first_record << 4 | count (om_bvh.cpp), not table indices
    // BVH4 collapsed from the BVH2 (same leaf table / records / always2)
    const OmBvh4Node* b4nodes;
    const OmBvh4NodeH* b4h;       // the same tree breadth-first with half-precision boxes (n_b4nodes nodes)
    uint32_t n_b4nodes;
    uint32_t b4_lds_bytes;        // node bytes when they fit the LDS budget, else 0 (global nodes)
    uint32_t b4_stack;            // lane-stack entries: 3 per level + 3 for the unconditional pushes
};

struct OmCamDev {
    float origin[3], horizontal[3], vertical[3], llc_minus_origin[3];
    float u[3], v[3];
    float lens_radius;
};

struct OmParamsDev {
    uint32_t width, height, spp_total, sample_count, max_depth, march_steps, adaptive;
    float tmin, tmax, wf_m1, hf_m1;   // (W-1), (H-1) as f32
    uint64_t skey;                     // mix64(seed + K) (om-rng v2 path key)
    uint32_t n_pixels;                 // pixels this launch covers
    uint32_t tiles_x;                  // 8x8 tiles per row (full-frame mapping)
    uint32_t progress;                 // 1: add credited samples to counters[OMC_PROGRESS] (om_progress)
};

// Counter slots (om_counters order); OMC_PROGRESS (the live progress word, om_progress) sits
// after them and is not cleared by om_reset_counters
enum { OMC_SAMPLES = 0, OMC_SEGMENTS, OMC_PRIM_TESTS, OMC_PRE_TESTS, OMC_MARCH, OMC_CREDITED, OMC_N };
enum { OMC_PROGRESS = OMC_N, OMC_SLOTS };
