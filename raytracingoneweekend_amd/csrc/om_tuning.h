// om_tuning.h — the wavefront pipeline's tunable sizes.  These
// are numbers, not code variants: every value renders the same bits (results are keyed by slot
// and (pixel, sample)), and tools/ablate.sh sweeps them by -D.  The measurements behind each
// default are in DESIGN.md; the code variants that measured slower are gone (git history and
// DESIGN.md §8 keep their numbers).
#pragma once

// Workgroup = one queue segment.  512 lanes share one LDS copy of the BVH2 nodes between 8
// waves, so LDS stops capping occupancy, and 8 waves/SIMD (<= 64 VGPRs) hide the incoherent
// bounces' latency.  C1 (r01): 256/no hint 3770, 256/8 3671, 512/- 3802, 512/8 3929, 1024/8 3368.
#ifndef OM_WF_BLOCK
#define OM_WF_BLOCK 512
#endif
#ifndef OM_WF_WAVES
#define OM_WF_WAVES 8
#endif
// queue segments per tail workgroup
#ifndef OM_WF_TAIL_SPB
#define OM_WF_TAIL_SPB 2
#endif
// paths per batch: 2^OM_WF_MIN_PATHS_LOG2 (16 spp of 1080p), raised to OM_WF_BATCH_SPP samples of
// the frame for frames above 2M pixels, within 2^OM_WF_MAX_PATHS_LOG2
#ifndef OM_WF_MAX_PATHS_LOG2
#define OM_WF_MAX_PATHS_LOG2 27
#endif
#ifndef OM_WF_BATCH_SPP
#define OM_WF_BATCH_SPP 16
#endif
#ifndef OM_WF_MIN_PATHS_LOG2
#define OM_WF_MIN_PATHS_LOG2 25
#endif
// A BVH2 too big for LDS (S-10k: 107 KB of half nodes) stages its breadth-first prefix, up to this
// many bytes of nodes, into LDS; deeper nodes are read through L2 (0 = every node from L2).  C3 with
// half nodes (r04_ab5/ab6): 8 / 12 / 16 / 20 / 24 / 28 KB -> 4113 / 4137 / 4135 / 4067 / 4069 / 3676.
#ifndef OM_WF_HYB_BYTES
#define OM_WF_HYB_BYTES 16384
#endif
// The same for the half-precision 4-wide tree (OM_KERNEL_BVH4 on a tree too big for LDS, §5.7).
// C3 (r05_b4h): 0 / 4 / 8 / 12 KB -> 4028 / 3943 / 3895-3918 / 3918 Msamples/s: lanes whose node
// is in LDS and lanes whose node is not run both loads, so every node comes through L1/L2.
#ifndef OM_WF_HYB4_BYTES
#define OM_WF_HYB4_BYTES 0
#endif
// k_march refills its idle lanes once at least this many of a wave's 64 wait
#ifndef OM_WF_REFILL
#define OM_WF_REFILL 16
#endif
// marched tail: a wave shades its ended marches once this many of its lanes wait (1 = at once).
// r04's sweep ran with a ballot that made every value behave as 1; with the ballots
// fixed (r05_p1, C2, two runs each): 1 / 8 / 16 -> 3422, 3389 / 3407, 3384 / 3377, 3360: no gain, 1.
#ifndef OM_WF_TAIL_SHADE
#define OM_WF_TAIL_SHADE 1
#endif
// marched tail: march steps per check, and the refill threshold (k_march's by default)
// C2 (r04_tmu, r04_tmu2, two runs each): 4 / 8 / 12 / 16 / 24 / 32 -> 3105 / 3275, 3279 / 3316, 3305 /
// 3333, 3349, 3361, 3366 / 3399, 3426 / 3399, 3387; refill 8 / 16 / 32 -> 3205, 3200 / 3275, 3279 / 3226, 3247
#ifndef OM_WF_TAIL_UNROLL
#define OM_WF_TAIL_UNROLL 24
#endif
// marched tail: waves per SIMD requested (8: 64 VGPRs, the 24-step loop spills 32 B per lane)
#ifndef OM_WF_TAIL_MARCH_WAVES
#define OM_WF_TAIL_MARCH_WAVES 8
#endif
#ifndef OM_WF_TAIL_REFILL
#define OM_WF_TAIL_REFILL OM_WF_REFILL
#endif
// marched worlds: first bounce run by the lane-refilling tail (0: the camera paths too; DESIGN.md
// §5.8).  C2 T = 12 / 6 / 4 / 3 / 2 / 1 -> 2906 / 3064 / 3081 / 3077 / 3209 / 3274 Msamples/s (r04_sw1-
// sw3, means of two runs); on the tuned tail T = 0 / 1 -> 2843, 2916 / 3425, 3413 (r04_q3)
#ifndef OM_WF_TAIL_MARCHED
#define OM_WF_TAIL_MARCHED 1
#endif
// k_march: march steps per refill check (the check costs three ballots and its branches).
// C2 (r03_v16/v17): 1 / 2 / 4 / 6 / 8 steps -> 2500 / 2587 / 2650 / 2661 / 2682 Msamples/s.
#ifndef OM_MARCH_UNROLL
#define OM_MARCH_UNROLL 8
#endif
// Adaptive calls: the live pixels are dealt to the streams by 64-entry chunks of the
// call's pixel list, and each stream renders ITS pixels in at most OM_WF_ADAPTIVE_BATCHES batches per
// call, from a live list its own k_accumulate compacts (ThreadPixels, render_thread.rs:68-102).  A
// batch's sample count is planned on the device from the stream's live count c: enough samples to
// give 2^OM_WF_ADAPTIVE_PATHS_LOG2 paths (c x b), at least an even share of the call's remaining
// samples over the batches left, at most the remainder.
#ifndef OM_WF_ADAPTIVE_BATCHES
#define OM_WF_ADAPTIVE_BATCHES 3
#endif
#ifndef OM_WF_ADAPTIVE_PATHS_LOG2
#define OM_WF_ADAPTIVE_PATHS_LOG2 22
#endif
// the queue capacity an adaptive call may raise its forced even share to (more batches beyond it)
#ifndef OM_WF_ADAPTIVE_CAP_LOG2
#define OM_WF_ADAPTIVE_CAP_LOG2 26
#endif
// tail threshold for adaptive batches (the per-bounce launches of a light batch are latency-bound)
#ifndef OM_WF_ADAPTIVE_TAIL
#define OM_WF_ADAPTIVE_TAIL 8
#endif
// Queue segments (= bounce workgroups) per CU: OM_WF_LANES_PER_CU / OM_WF_BLOCK; marched worlds
// and BVH2s read through L2 use the WIDE count.
#ifndef OM_WF_LANES_PER_CU
#define OM_WF_LANES_PER_CU 4096
#endif
#ifndef OM_WF_LANES_PER_CU_WIDE
#define OM_WF_LANES_PER_CU_WIDE 8192
#endif
// k_accumulate: samples whose loads are issued together before their adds in sample order
#ifndef OM_ACC_GROUP
#define OM_ACC_GROUP 8
#endif
// BVH2 f32 nodes staged whole in LDS: bytes between consecutive nodes (64 = packed).  A wave's
// node reads are ds_read_b128/b96 at random nodes; at a 64-B stride word k of every node falls
// in one of 4 (b128) / 2 (b96) bank slots, at 80 B in one of 16 / 8 (r06, VERDICT r05 #1b).
// C1 (r06_ab1, r06_ab2): 80 -> 7128, 7118 / 6902, 6911 vs 64 -> 7077, 7107 / 6863, 6874 Msamples/s.
#ifndef OM_B2_NODE_STRIDE
#define OM_B2_NODE_STRIDE 80
#endif
