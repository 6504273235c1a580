// om_world.h — host HittableList and its frozen, device-ready image.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"
#include "om_hostmath.h"
#include "om_layout.h"

namespace om {

struct AffinePrim { Mat4 l2w, w2l; om_material mat; };              // Sphere / Cube (traced.rs:13-19, 229-235)
struct BaryPrim {                                                     // Barycentric<BT> (traced.rs:118-131)
    Vec3 origin, u; float u_length; Vec3 v; float v_length; Vec3 uxv, uxvxu; Mat3 base_inv; Vec3 v_in_base; om_material mat;
};
struct PlanePrim { Vec3 center, normal; om_material mat; };          // InfinitePlane (traced.rs:77-82)
struct MSpherePrim { Vec3 center; float radius; om_material mat; };  // marched.rs:50-54
struct MBoxPrim { Vec3 center, sizes; om_material mat; };            // marched.rs:79-83
struct MTorusPrim { Mat4 l2w_tr, w2l_tr; Vec4 l2w_s, w2l_s; Vec3 sizes; om_material mat; };  // marched.rs:105-113
// a user marched object (Arc<dyn Marched>, hits.rs:96-100): MarchedTorus's transform + an SDF program
struct MSdfPrim { MTorusPrim xf; std::vector<OmSdfOp> ops; om_material mat; };

enum PrimKind { K_SPHERE = 0, K_CUBE = 1, K_TRI = 2, K_PLANE = 3, K_PARA = 4, K_MSPHERE = 5, K_MBOX = 6, K_MTORUS = 7,
                K_MSDF = 8, K_N = 9 };

// Frozen image of a world: arrays laid out exactly as they are copied to HBM.
struct FrozenWorld {
    std::vector<OmAffineTest> sph_test, cube_test;
    std::vector<OmAffineHit> sph_hit, cube_hit;
    std::vector<OmBound> sph_bound, cube_bound;
    std::vector<OmBary> tri, para;
    std::vector<OmPlane> plane;
    std::vector<OmMSphere> msph;
    std::vector<OmMBox> mbox;
    std::vector<OmMTorus> mtor;
    std::vector<OmMSdf> msdf;          // user marched objects
    std::vector<OmSdfOp> msdf_ops;     // their programs, back to back
    std::vector<OmMaterial> mats;      // by global index
    std::vector<uint64_t> bloom;       // by obj id
    std::vector<OmBvhNode> bvh;
    std::vector<uint32_t> bvh_prims;   // global indices
    std::vector<uint32_t> always;      // global indices tested outside the BVH
    std::vector<OmSkipNode> snodes;    // stackless BVH (affine prims only)
    std::vector<OmAffineTest> srecs;   // its records in leaf order
    std::vector<uint32_t> always2;     // prims outside the stackless BVH
    std::vector<OmAlwaysRec> always2_rec;  // the same, with their conservative boxes
    std::vector<float> srec_box;       // per srec: inflated box lo xyz, hi xyz (primary-ray tile lists)
    std::vector<OmBvh2Node> b2nodes;   // compressed BVH2 (same leaves/records as snodes)
    std::vector<OmBvh2NodeH> b2h;      // the same nodes with half-precision boxes rounded outward (device)
    std::vector<uint32_t> b2leaves;    // its leaf table: (first_record << 8) | count
    uint32_t b2_depth = 0;             // its depth (stack bound)
    uint32_t b2_direct = 0;            // 1: leaf child codes carry OM_LEAF | first_record << 4 | count (no table read)
    std::vector<OmBvh4Node> b4nodes;   // 4-wide tree collapsed from b2nodes (leaf codes index b2leaves)
    std::vector<OmBvh4NodeH> b4h;      // the same tree breadth-first, half-precision boxes rounded outward
    uint32_t b4_depth = 0;             // its depth
    uint32_t counts[K_N];
    uint32_t offsets[K_N + 1];         // global index offset per kind, offsets[K_N] = total
};

uint64_t bloom_hash(uint64_t id);      // utils.rs:94-107

}  // namespace om

struct om_world {
    std::vector<om::AffinePrim> spheres, cubes;
    std::vector<om::BaryPrim> triangles, parallelograms;
    std::vector<om::PlanePrim> planes;
    std::vector<om::MSpherePrim> msph;
    std::vector<om::MBoxPrim> mbox;
    std::vector<om::MTorusPrim> mtor;
    std::vector<om::MSdfPrim> msdf;
    void freeze(om::FrozenWorld& fw) const;
};
