/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into libvccl; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * CPU restatement of VCCL's bucket-reduction semantics (the reference is CUDA
 * and cannot be compiled here: no nvcc):
 *   - per-element ops      reduce_kernel.h:174-323 (Apply_Reduce)
 *   - preOp / postOp       reduce_kernel.h:410-688 (PreMulSum, SumPostDiv)
 *   - op-arg encoding      enqueue.cc:2217-2310 (hostToDevRedOp)
 *   - signed->unsigned     generate.py:129-137 (equivalent_primary)
 *   - fold order           common_kernel.h:84-152 (reduceCopyPacks)
 *   - ring fold order      all_reduce.h:32-82, reduce_scatter.h:33-54
 *
 * Parity status: the dispatch/type table is pinned against the reference's own
 * generate.py output (tests/golden/gen_functable.py).  The fp16/bf16 arithmetic
 * comes from CUDA's cuda_fp16.h / cuda_bf16.h intrinsics, which are not vendored
 * in /root/reference and not present in this image, and no reference-produced
 * fixture exists.  The ARITHMETIC is pinned to the reference's own fallback
 * expressions (reduce_kernel.h:276-277, 285, 294-296: widen, one binary32 op,
 * round RN-even), evaluated by independent IEEE-754 implementations (numpy,
 * torch-CPU) in tests/golden/reduce_golden.npz; the intrinsic branch gives the
 * same bits by the innocuous-double-rounding bound (24 >= 2p + 2 for binary16
 * and bfloat16).  Open: FTZ of subnormals, NaN payloads.
 */
#ifndef VCCL_ORACLE_REDUCE_REF_H_
#define VCCL_ORACLE_REDUCE_REF_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ncclDataType_t values (nccl.h.in:239-252) */
enum { R_I8 = 0, R_U8, R_I32, R_U32, R_I64, R_U64, R_F16, R_F32, R_F64, R_BF16, R_F8E4M3, R_F8E5M2 };
/* ncclDevRedOp_t values (src/include/device.h:34-38) */
enum { R_SUM = 0, R_PROD, R_MINMAX, R_PREMULSUM, R_SUMPOSTDIV };
/* ncclRedOp_t values (nccl.h.in:221-236) */
enum { R_OP_SUM = 0, R_OP_PROD, R_OP_MAX, R_OP_MIN, R_OP_AVG };

int ref_type_size(int type);
/* hostToDevRedOp (enqueue.cc:2217-2310): returns 0 on success. */
int ref_host_to_dev_redop(int op, int type, int nranks, int* devOp, uint64_t* opArg);

/* Bit-exact conversions (IEEE-754 binary16 / bfloat16, round-to-nearest-even,
 * subnormals kept, NaN stays NaN). */
float ref_f16_to_f32(uint16_t h);
uint16_t ref_f32_to_f16(float f);
float ref_bf16_to_f32(uint16_t h);
uint16_t ref_f32_to_bf16(float f);
/* OCP FP8 E4M3 ("fn", bias 7, max 448, NaN S.1111.111) and E5M2 (bias 15,
 * max 57344).  Widening is exact; narrowing is __nv_cvt_float_to_fp8(x,
 * __NV_SATFINITE, fmt): RN-even, |x| past max finite (infinity included) ->
 * max finite, NaN -> 0x7f. */
float ref_fp8_to_f32(int type, uint8_t b);
uint8_t ref_f32_to_fp8(int type, float f);

/* Element primitives on raw bits (value in the low sizeof(T) bytes). */
uint64_t ref_reduce1(int devOp, int type, uint64_t opArg, uint64_t a, uint64_t b);
uint64_t ref_preop1(int devOp, int type, uint64_t opArg, uint64_t a);
uint64_t ref_postop1(int devOp, int type, uint64_t opArg, uint64_t a);

/* reduceCopy (common_kernel.h:208-285):
 *   dst_j[i] = postOp( preOp_0(src_0[i]) (+) preOp_1(src_1[i]) (+) ... )
 * preOp applies to sources s < preOpSrcs with preOpArgs[s]; fold is left to
 * right (acc = acc (+) src_s).  nthreads > 1 splits the range over pthreads. */
void ref_reduce_copy(int devOp, int type, uint64_t redArg, const uint64_t* preOpArgs,
                     int preOpSrcs, int postOp, int nSrcs, const void* const* srcs,
                     int nDsts, void* const* dsts, size_t nElts, int nthreads);

/* Ring fold of one element range (all_reduce.h:42-64 / reduce_scatter.h:39-53).
 * inputs[k] = the input of the rank at ring index k.  owner[i] = ring index of
 * the rank that finishes element i.  The fold starts at ring index owner+1
 * (a send of its preOp'd input), each next rank computes preOp(own) (+) recv,
 * and the owner applies postOp:  x_o (+) (x_{o-1} (+) (... (+) x_{o+1})). */
void ref_ring_fold(int devOp, int type, uint64_t redArg, int preOp, int nranks,
                   const void* const* inputs, const int32_t* owner, void* out,
                   size_t nElts);

/* Chain ("tree" on one node, graph/connect.cc:64-65) fold used by the LL
 * tree all-reduce (all_reduce.h:148-229, prims_ll.h:258-266): the leaf at
 * chain position n-1 sends, each position p computes peer (+) own going up,
 * the root (position 0) applies postOp.  inputs[p] = rank at chain pos p. */
void ref_chain_fold(int devOp, int type, uint64_t redArg, int preOp, int nranks,
                    const void* const* inputs, void* out, size_t nElts);

/* Host-core baseline (cpu_bench.c; bench.py's cpu_baseline leg only): the
 * config-2 shape (f32 d = a + b over n elements) on `nthreads` persistent
 * workers pinned to cpus[t] (NULL = unpinned), buffers first-touched by
 * their owners.  run returns 1 when the result checks bit-exactly. */
int ref_cpu_bench_alloc(size_t n, int nthreads, const int* cpus, void** a, void** b, void** d);
int ref_cpu_bench_run(void* a, void* b, void* d, size_t n, int nthreads, const int* cpus,
                      double seconds, long* iters, double* elapsed);
void ref_cpu_bench_free(void* a, void* b, void* d, size_t n);
/* One rank's share of an n-rank ring all-reduce as host work: an nsrc-source
 * sum over m elements of `type` (f32 7, f16 6 or bf16 9) into one shard, then
 * a copy of ncopy elements (the gather; 0 = none).  bufs[nsrc + 3]: sources,
 * shard, copy source, copy destination.  run returns 1 when the shard (folded
 * left to right with ref_reduce1) and the copy check bit-exactly. */
int ref_cpu_bench_rank_alloc(size_t m, int nsrc, size_t ncopy, int type, int nthreads, const int* cpus,
                             void** bufs);
int ref_cpu_bench_rank_run(void** bufs, size_t m, int nsrc, size_t ncopy, int type, int nthreads,
                           const int* cpus, double seconds, long* iters, double* elapsed);
void ref_cpu_bench_rank_free(void** bufs, size_t m, int nsrc, size_t ncopy, int type);

#ifdef __cplusplus
}
#endif
#endif
