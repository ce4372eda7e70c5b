// grs_config.h — compile-time constants shared by host and device code.
//
// Replaces the reference's shared GLSL/C++ constant headers
// (Shaders/ParallelSort/ParallelSortConstants.comp:17-24,
//  Shaders/ComputeHeaders/SsboBufferBindings.comp:19-22,
//  Shaders/ComputeHeaders/UniformLocations.comp:24-38), which #define one 512-thread
// work group and 1024 items per scan group for a 32 x 1-bit LSD sort.  Here the digit
// width is a template parameter (4 or 8 bits) and one onesweep tile holds
// GRS_BLOCK x ITEMS keys; buffer bindings and uniform locations have no equivalent
// (kernel arguments carry the pointers).
#pragma once

#include <stdint.h>

#define GRS_WAVE 64                 // CDNA wavefront width (never 32)
#define GRS_BLOCK 512               // threads per onesweep workgroup (8 waves)
#define GRS_HIST_BLOCK 256

// Largest element count one device sort call accepts.  Look-back words hold counts + 1
// (grs_pass.hpp), so every prefix fits 32 bits; the bound keeps tile arithmetic
// (tile * TILE + TILE) inside 32 bits for every tile shape (TILE < 2^16).
#define GRS_MAX_N 0xFFFF0000ull

// Bounded spins (look-back): give up after this many polls and raise the error word.
#ifndef GRS_SPIN_LIMIT
#define GRS_SPIN_LIMIT (1u << 22)
#endif
// Key-range partition (multi-GPU exchange): at most this many splitters -> 16 buckets.
#define GRS_MAX_SPLITTERS 15

// Predecessor tiles polled per look-back step (loads in flight per digit thread).
#ifndef GRS_LB_WIN
#define GRS_LB_WIN 8
#endif

// Two-level look-back: tiles per group, and groups polled per group-level step.
#ifndef GRS_LB_GROUP
#define GRS_LB_GROUP 8
#endif
#ifndef GRS_LB_GWIN
#define GRS_LB_GWIN 8
#endif
// the same for two-round (XL) tiles, whose keys stay live in VGPRs beside the window
#ifndef GRS_LB_GWIN_XL
#define GRS_LB_GWIN_XL 4
#endif

// XCDs of an MI355X (8 x 32 CUs, each XCD with its own L2): ticket counters are XCD-strided.
#define GRS_XCDS 8

// Layout of the per-sorter control block (uint32 words), zeroed once per sort call.
//   [0, GRS_CTRL_HIST_WORDS)           digit histograms, [pass][256] (the upfront kernel's)
//   GRS_CTRL_TICKETS + pass * 8        per-pass tile ticket counter
//   GRS_CTRL_ERROR                     nonzero = a bounded spin timed out; [1], [2] the pass's
//                                      debug words (grs_pass.hpp PassDebug)
//   GRS_CTRL_PLAN + pass               the LSD sort's pass plan (grs_pass_plan), written each call
#define GRS_MAX_PASSES 16               // u64 keys at 4-bit digits
#define GRS_HIST_PASS_STRIDE 256
#define GRS_CTRL_HIST_WORDS (GRS_MAX_PASSES * GRS_HIST_PASS_STRIDE)
#define GRS_CTRL_TICKETS GRS_CTRL_HIST_WORDS
#define GRS_CTRL_ERROR (GRS_CTRL_TICKETS + GRS_MAX_PASSES * GRS_XCDS)
#define GRS_CTRL_PLAN (GRS_CTRL_ERROR + 16)
#define GRS_CTRL_WORDS (GRS_CTRL_PLAN + GRS_MAX_PASSES)   // multiple of 4 words (16-B memset)
