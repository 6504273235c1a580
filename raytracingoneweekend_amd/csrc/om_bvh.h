// om_bvh.h — host BVH builder over the bounded traced primitives.
//
// The reference has no acceleration structure: FrozenHittableList::hit tests
// every traced object in type order (hits.rs:274-285).  Its result is the
// smallest accepted root, ties going to the later object.  The BVH only decides
// WHICH exact tests run; boxes are conservative, and the kernel applies the same
// tie rule, so the closest hit is bit-identical to brute force.
#pragma once
#include "om_world.h"

namespace om {
void build_bvh(const om_world& w, FrozenWorld& fw);
// the half-precision node planes (OmBvh2NodeH): a half's exact value, and the half that holds a
// float plane on the outside (lo: the largest half <= x, hi: the smallest half >= x; NaN -> the
// infinite plane, so a NaN box culls nothing)
float half_value(uint16_t h);
uint16_t half_out(float x, bool up);
void build_skip_bvh(const om_world& w, FrozenWorld& fw);
}
