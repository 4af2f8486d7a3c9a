/*
 * cio_diag.h -- every compile-time A/B and diagnostic switch of the kernels,
 * in one place.  A product build (`make`) defines none of them, so the
 * defaults below ARE the shipped kernels.  A/B builds override one with
 * `make ablib VAR=name DEFS=-DX=v` (or ablib_sha1), which writes a separate
 * library under chunkio_amd/lib/ab/ for tools/ab_lib.py / tools/gpu_ab.sh.
 *
 * "Diagnostic" switches compute WRONG results on purpose (they remove work
 * to price it); they exist only to measure, never to ship.
 */
#ifndef CIO_DIAG_H
#define CIO_DIAG_H

/* ---- crc32_gpu.hip ------------------------------------------------------ */

/* Diagnostic (round-3 probe, rejected): CIO_DIAG_RS_DYN compiles
 * read_stream_dyn_kernel, the read-only stream with a dynamically claimed
 * tail, selected at run time by CIO_GPU_RS_DYN="pool_permille,U,NC"
 * (tools/rs_dyn_probe.py; `make ablib VAR=rsdyn DEFS=-DCIO_DIAG_RS_DYN`).
 * Not in the product library. */

/* Diagnostic: lanes read 16 slice / 4 shift table replicas instead of 32 / 8
 * (the 2-way bank conflicts of a two-workgroups-per-CU layout, priced at
 * today's occupancy).  Correct results, slower kernel. */
#ifndef CIO_DIAG_HALF_REPLICAS
#define CIO_DIAG_HALF_REPLICAS 0
#endif

/* Diagnostic: the stream kernel computes on register data instead of HBM
 * loads (compute-only time; wrong CRCs). */
#ifndef CIO_ABLATE_LOADS
#define CIO_ABLATE_LOADS 0
#endif

/* Diagnostic: skip the arrival/fold step of split chunks (prices the tail;
 * wrong CRCs for split chunks).  2: also skip the arrival descriptors' loads
 * at kernel start (prices their share of the start-up). */
#ifndef CIO_DIAG_NO_ARRIVAL
#define CIO_DIAG_NO_ARRIVAL 0
#endif

/* Diagnostic: 1 = finished waves stay resident ~5 us before exiting, 2 = they
 * wait for their workgroup (correct results). */
#ifndef CIO_DIAG_TAIL
#define CIO_DIAG_TAIL 0
#endif

/* A/B: chunks whose pieces all lie in one workgroup fold through LDS (1,
 * shipped) or through the global arrival counters (0). */
#ifndef CIO_LDS_FOLD
#define CIO_LDS_FOLD 1
#endif

/* A/B: the issue-ahead stream kernel peels each wave's last step off its
 * loop so that step issues no refill (1), or refills unconditionally (0). */
#ifndef CIO_AHEAD_PEEL
#define CIO_AHEAD_PEEL 1
#endif

/* Small-chunk kernel.  A/B: chunks in flight per wave (1 shipped, 2).
 * Diagnostic bit mask: 1 = no lane multiply, 2 = no LDS CRC (wrong CRCs). */
#ifndef CIO_SMALL_SLOTS
#define CIO_SMALL_SLOTS 1
#endif
#ifndef CIO_SMALL_EXP
#define CIO_SMALL_EXP 0
#endif

/* Alignment of a chunk's virtual start for chunks longer than one 4 KiB
 * step: 128 (one L2 line, shipped from round 5) or 16 (rounds 1-4).  At 128
 * every 1 KiB row of such a chunk is line-aligned, so consecutive rows and
 * steps never share a line; the head (up to 127 bytes of the neighbour) is
 * zeroed in registers as the 16-byte head always was.  At 16, a chunk at an
 * offset that is not a multiple of 128 re-fetched the line each step boundary
 * shares (cfg3, 16-byte packed: 1.024x the algorithmic bytes; at 128:
 * 1.0004x, profiles/r05/cfg3_traffic/).  Chunks of at most one step keep 16
 * (they stay on the small-chunk kernel). */
#ifndef CIO_HEAD_ALIGN
#define CIO_HEAD_ALIGN 128
#endif

/* Small-chunk kernel, L64 layout (CIO_GPU_L64=1): the lane's final multiply by
 * x^(8 * 64 (63 - L)) as 8 nibble-table lookups in the LDS the L64 layout
 * leaves free (the 32 KiB shift-table region: [nibble position j][nibble]
 * [lane] words, built per workgroup from the lane's register matrix) instead
 * of 32 bit-select + fused and-xor instructions. */
#ifndef CIO_SMALL_NIBFOLD
#define CIO_SMALL_NIBFOLD 0
#endif

/* ---- sha1_gpu.hip -------------------------------------------------------- */

/* A/B: blocks handed over per barrier, schedule waves, chunks per workgroup
 * of the wide geometry. */
#ifndef CIO_SHA1_GROUP
#define CIO_SHA1_GROUP 4
#endif
#ifndef CIO_SHA1_SCHED_WAVES
#define CIO_SHA1_SCHED_WAVES 1
#endif
#ifndef CIO_SHA1_CHAINS
#define CIO_SHA1_CHAINS 32
#endif
/* A/B: the round wave issues the next block's 20 row reads after this many
 * rows (x 4 rounds) of the current block; 0 = before it (shipped). */
#ifndef CIO_SHA1_READ_AT
#define CIO_SHA1_READ_AT 0
#endif
/* A/B: blocks per barrier of the 8-chunk geometry (cfg5's). */
#ifndef CIO_SHA1_GROUP8
#define CIO_SHA1_GROUP8 8
#endif

/* A/B: 1 drops the asm anchor that keeps each block's rounds ahead of the
 * next block's row reads (correct results, slower). */
#ifndef CIO_SHA1_NO_ANCHOR
#define CIO_SHA1_NO_ANCHOR 0
#endif

/* Timing-only ablations of the SHA-1 kernel (WRONG digests on purpose; A/B
 * builds for tools/sha1_ab.py --diag, profiles/r06/sha1_attribution/):
 * NOREAD: the round wave reads two blocks' rows once and reuses them (no LDS
 * row reads in the loop); NOBAR: no hand-over barriers; NOSCHED: the schedule
 * wave exits at once (use with NOBAR). */
#ifndef CIO_SHA1_DIAG_NOREAD
#define CIO_SHA1_DIAG_NOREAD 0
#endif
#ifndef CIO_SHA1_DIAG_NOBAR
#define CIO_SHA1_DIAG_NOBAR 0
#endif
#ifndef CIO_SHA1_DIAG_NOSCHED
#define CIO_SHA1_DIAG_NOSCHED 0
#endif

/* Diagnostic: per-workgroup shader-clock records of the round loop, read back
 * by cio_sha1_diag_clock (tools/sha1_clock.py).  Correct results. */
#ifndef CIO_SHA1_CLOCK_DIAG
#define CIO_SHA1_CLOCK_DIAG 0
#endif

/* ---- host_pipeline.hip ---------------------------------------------------- */

/* A/B: staging slots per host pipeline. */
#ifndef CIO_PIPE_SLOTS
#define CIO_PIPE_SLOTS 3
#endif

#endif /* CIO_DIAG_H */
