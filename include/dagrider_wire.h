/*
 * dagrider_wire.h -- DRW1 capture format reader (C ABI).
 *
 * The reference ships vertices between processes as Go values over channels
 * (bcastMsg, process/transport.go:13-17, carrying vertex, process/process.go:26-31)
 * and has no on-disk form.  A DRW1 capture stores a [][]vertex as exactly the
 * flat arrays dr_append_rounds_lists takes (dag_rider_amd/wire.py writes them;
 * go/dagridergpu/wire.go too), so any caller can replay a captured run into a
 * device mirror without Python.
 *
 * Layout (little-endian): magic "DRW1", u32 nrounds, u32 nslots; six arrays in
 * dr_append_rounds_lists order -- slot_off u32[nrounds+1], slot_id i32[2*nslots],
 * strong_off u32[nslots+1], strong_ids i32[2*Es], weak_off u32[nslots+1],
 * weak_ids i32[2*Ew] -- each preceded by its u64 element count; then
 * block_off u64[nslots+1] and the block bytes.
 *
 * Every size and offset is checked before anything is used (the append trusts
 * its arrays as raw pointers): a truncated or corrupt buffer gives DR_E_INVAL.
 */
#ifndef DAGRIDER_WIRE_H
#define DAGRIDER_WIRE_H
#include <stddef.h>
#include <stdint.h>

#include "dagrider_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Validate a capture; on DR_OK report its round and slot counts (either may be
 * NULL).  Host-only: needs no device. */
int dr_wire_check(const void *buf, size_t len, int32_t *nrounds, int32_t *nslots);

/* Append every round of the capture to the mirror (rounds [r0, r0+nrounds) with
 * r0 = dr_num_rounds(ctx); the capture's round ids are its own).  Errors: those
 * of dr_wire_check (DR_E_INVAL) and of dr_append_rounds_lists. */
int dr_wire_append(dr_ctx *ctx, const void *buf, size_t len);

/* Block payload of slot i (vertex.block, never read by the hot path): pointer
 * into buf and its length, or DR_E_INVAL. */
int dr_wire_block(const void *buf, size_t len, int64_t slot, const uint8_t **data, size_t *n);

#ifdef __cplusplus
}
#endif
#endif
