/*
 * ambrycrc.h -- C ABI of libambrycrc, the MI355X (gfx950) CRC-32 engine for
 * Ambry's per-record / per-chunk checksum path.
 *
 * Function: CRC-32/ISO-HDLC (reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF),
 * bit-exact with com.github.ambry.utils.Crc32 and java.util.zip.CRC32.
 *
 * Value convention: zlib-style *finalized* CRCs. A running CRC starts at 0 and
 * ambrycrc_update(crc, p, n) returns the value Checksum.getValue() would report
 * after update(p, 0, n) on a checksum whose getValue() was `crc`. Ambry's
 * Crc32 keeps the bit-inverted register internally (Crc32.java:37-52); its
 * register equals ~value.
 *
 * Ownership: the caller owns every buffer. The library never frees caller
 * memory and never retains a pointer past the call (for *_dev functions: past
 * completion of the work it enqueued on the caller's stream). Device tables
 * and the default workspace belong to a per-device context created by
 * ambrycrc_init().
 *
 * Errors: every int-returning function returns AMBRYCRC_OK (0) or a negative
 * code; nothing aborts or throws across the ABI. A CRC *mismatch* is data
 * (ambrycrc_verify_dev's flags), not an error.
 *
 * Threading: the host functions are reentrant with no mutable global state.
 * The *_dev functions may be called from several host threads; each call
 * enqueues on the caller's stream. With d_ws == NULL a call uses the default
 * workspace of its stream (one per stream, so calls on different streams never
 * share one); a caller workspace (ambrycrc_workspace_bytes) must not be used by
 * two calls whose work overlaps. Under stream capture (a HIP graph) a call with
 * d_ws == NULL uses its stream's default workspace as an earlier uncaptured call
 * on that stream sized it, and returns AMBRYCRC_EINVAL if that is too small.
 */
#ifndef AMBRYCRC_H
#define AMBRYCRC_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h> /* hipStream_t */

#ifdef __cplusplus
extern "C" {
#endif

#define AMBRYCRC_OK 0
#define AMBRYCRC_EINVAL (-1)   /* bad argument (null pointer, bad size, alignment) */
#define AMBRYCRC_EHIP (-2)     /* a HIP runtime call failed */
#define AMBRYCRC_ENOMEM (-3)   /* device or pinned-host allocation failed */
#define AMBRYCRC_ENOINIT (-4)  /* ambrycrc_init() not called for the current device */
#define AMBRYCRC_ENODEV (-5)   /* no usable gfx950 device */
#define AMBRYCRC_ECOMM (-6)    /* RCCL unavailable, or a collective / communicator call failed */
#define AMBRYCRC_EPROBE (-7)   /* ambrycrc_init: this library is an A/B timing build (wrong CRCs) and
                                  AMBRYCRC_ALLOW_PROBE=1 is not set */

/* ---------------------------------------------------------------- lifecycle */

/* Create the context of `device` (LDS table image in HBM, default workspace).
 * Idempotent. Replaces nothing in the reference: Ambry's Crc32 tables are static
 * (Crc32.java:154-179); this is where their device copy is made. */
int ambrycrc_init(int device);

/* Release every context. Outstanding work must have completed. */
int ambrycrc_shutdown(void);

/* Static, human-readable description of an error code. */
const char* ambrycrc_strerror(int code);

/* Library version string: "ambrycrc <semver> gfx950", followed by " ab-probe-build" and
 * " AMBRY_<KNOB>=<value>" for every compile-time A/B knob that differs from the product default
 * (ambry_amd/csrc/build_knobs.h). The product build reports neither. */
const char* ambrycrc_version(void);

/* ------------------------------------------------- host streaming primitives */

/* Continue a finalized CRC over n host bytes (CPU; for the small, per-record
 * updates that cannot amortize a device round trip).
 * Replaces Crc32.update(byte[],int,int) (ambry-utils/.../utils/Crc32.java:55-98),
 * Crc32.update(ByteBuffer) (:100-143) and java.util.zip.CRC32.update as used by
 * CrcInputStream.read/updateCrc (ambry-utils/.../utils/CrcInputStream.java:46-71). */
uint32_t ambrycrc_update(uint32_t crc, const void* p, size_t n);

/* Continue over a gather list of n buffers in order (one call for a Netty CompositeByteBuf's
 * nioBuffers()): the loop of PutOperation.PutChunk.verifyCRC (ambry-router/.../
 * PutOperation.java:2041-2043), `for (ByteBuffer b : buf.nioBuffers()) crc.update(b)`.
 * Equals n successive ambrycrc_update calls; a NULL pointer with length 0 is allowed. */
uint32_t ambrycrc_update_iov(uint32_t crc, const void* const* ptrs, const size_t* lens, size_t n);

/* n independent host chunks on `threads` CPU threads (0 = one per CPU this process may run on):
 * out[i] = crc32(crc_in ? crc_in[i] : 0, ptrs[i], lens[i]), with the loop ambrycrc_update runs.
 * The many-record CPU batch for bytes that live in host memory and are not going to the GPU
 * anyway (a GET's FileChannel read, a PUT's Netty buffers: DESIGN.md §5 "the CPU wins"); the
 * reference runs one Crc32 per record on the calling thread (Crc32.java:55-98). Synchronous. */
int ambrycrc_batch_cpu(const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in, uint32_t* out, size_t n,
                       int threads);

/* One byte: Crc32.update(int b) (Crc32.java:146-148). */
uint32_t ambrycrc_update_byte(uint32_t crc, int b);

/* Name of the CPU implementation ambrycrc_update runs: "vpclmul" (AVX-512
 * carry-less-multiply fold), "pclmul" (SSE fold) or "slice8" (the table loop of
 * Crc32.java:55-98). Chosen once per process from the CPU's features; the
 * environment variable AMBRYCRC_HOST_IMPL can lower it (tests, benches). Inputs
 * under 64 B always take slice8. No Java counterpart (HotSpot's CRC32 intrinsic
 * makes the same choice inside the JVM). */
const char* ambrycrc_host_impl(void);

/* crc(A||B) from crc(A), crc(B) and |B| (zlib crc32_combine semantics). No Java
 * counterpart in Ambry; it is what lets a chunk be split across lanes/GPUs and
 * lets a blob record's CRC be derived from the blob's (PutMessageFormatInputStream.java:116-120). */
uint32_t ambrycrc_combine(uint32_t crc1, uint32_t crc2, uint64_t len2);

/* CRC of n zero bytes continuing from crc (HardDeleteMessageFormatInputStream's
 * ZeroBytesInputStream records, ambry-messageformat/.../HardDeleteMessageFormatInputStream.java:58-124). */
uint32_t ambrycrc_zeros(uint32_t crc, uint64_t n);

/* ------------------------------------------------ device-resident batch path */

/* Bytes of device workspace a batch of n chunks needs. */
size_t ambrycrc_workspace_bytes(size_t n);

/* CRC-32 of n independent chunks in HBM:
 *   d_out[i] = crc32(d_crc_in ? d_crc_in[i] : 0, d_base + d_off[i], d_len[i]).
 * d_off/d_len/d_crc_in/d_out are device arrays; chunks may have any alignment
 * and length (0 included) and may overlap. Enqueued on `stream`; asynchronous.
 * d_ws/ws_bytes: optional workspace (>= ambrycrc_workspace_bytes(n)); NULL uses
 * the context's. Batch form of Crc32.update(ByteBuffer) + getValue() as the
 * router runs it per chunk (ambry-router/.../PutOperation.java:1700-1703 fill,
 * :2033-2054 verifyCRC) and of the blob-record CRC
 * (ambry-messageformat/.../MessageFormatRecord.java:1797-1832). */
int ambrycrc_batch_dev(const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len,
                       const uint32_t* d_crc_in, uint32_t* d_out, size_t n, void* d_ws, size_t ws_bytes,
                       hipStream_t stream);

/* As ambrycrc_batch_dev, then compare with d_expected: d_mismatch[i] = 1 iff the
 * CRC differs (either output pointer may be NULL; *d_mismatch_count is
 * incremented per mismatch, caller zeroes it). d_out may be NULL (internal).
 * Batch form of the `actualCRC != expectedCRC` checks of verify-on-read:
 * MessageFormatRecord.java:1184-1190, 1642-1646, 1823-1829; PutOperation.java:2040-2050. */
int ambrycrc_verify_dev(const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len,
                        const uint32_t* d_crc_in, const uint32_t* d_expected, uint32_t* d_out,
                        uint8_t* d_mismatch, uint32_t* d_mismatch_count, size_t n, void* d_ws,
                        size_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------- message-level verify (§8f) */

/* Per-message status bits of ambrycrc_verify_messages_dev (0 = every CRC matches). */
#define AMBRYCRC_MSG_HEADER_CRC (1u << 0)   /* header CRC (verifyHeader, MessageFormatRecord.java:1132-1145) */
#define AMBRYCRC_MSG_ENCKEY_CRC (1u << 1)   /* BlobEncryptionKey_Format_V1 (:1588-1600) */
#define AMBRYCRC_MSG_PROPS_CRC (1u << 2)    /* BlobProperties_Format_V1 (:1179-1195) */
#define AMBRYCRC_MSG_UPDATE_CRC (1u << 3)   /* Update_Format_V1..V3 (:1215-1420) */
#define AMBRYCRC_MSG_USERMETA_CRC (1u << 4) /* UserMetadata_Format_V1 (:1637-1649) */
#define AMBRYCRC_MSG_BLOB_CRC (1u << 5)     /* Blob_Format_V1..V3 (:1668-1833) */
#define AMBRYCRC_MSG_BAD_VERSION (1u << 8)  /* MessageFormatErrorCodes.UnknownFormatVersion: the header's, or a
                                               record's version (MessageFormatRecord.java:147-239) */
#define AMBRYCRC_MSG_BAD_LAYOUT (1u << 9)   /* HeaderConstraintError, or the message overruns the region */
#define AMBRYCRC_MSG_BAD_RECORD (1u << 11)  /* a record's own size field disagrees with its span in the header
                                               (encryption key, user metadata, blob: the stream would look for
                                               the CRC elsewhere), a blob type ordinal >= 2, a blob size >
                                               Integer.MAX_VALUE (the DataCorrupt / IOException cases of
                                               deserializeBlob*), or a record too short for its fields;
                                               BlobProperties: a SerDe version outside 1..5, a negative
                                               string size, a field past the span, or fields that end
                                               before it (BlobPropertiesSerDe.java:56-77 under
                                               MessageFormatRecord.java:1179-1195); Update: an unknown
                                               SubRecord.Type or fields that do not end at the CRC
                                               (:1217-1228, 1253-1266, 1388-1413) */

/* Bytes of device workspace ambrycrc_verify_messages_dev needs for m messages. */
size_t ambrycrc_messages_workspace_bytes(size_t m);

/* Verify every CRC of m PUT / update messages that start at d_msg_off[i] inside
 * [d_region, d_region + region_len): header (V1/V2/V3), encryption key, blob
 * properties, update, user metadata and blob records. d_status[i] gets the
 * AMBRYCRC_MSG_* bits (all corrupt records, not just the first: the reference's
 * deserializeBlobAll throws at the first, which is the lowest record bit set, with
 * UnknownFormatVersion when AMBRYCRC_MSG_BAD_VERSION is set for it). Besides the CRCs, each
 * record's version and size fields are checked against the header's record spans.
 * A corrupt header stops the message there, as verifyHeader does. d_msg_end[i]
 * (nullable) gets the offset one past the message, or 0 when unparseable.
 * Batch form of deserializeBlobAll's checks (MessageFormatRecord.java:257-303),
 * BlobStoreRecovery.recover (BlobStoreRecovery.java:43-110) and
 * ValidatingTransformer.transform (ValidatingTransformer.java:46-104). */
int ambrycrc_verify_messages_dev(const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off, size_t m,
                                 uint32_t* d_status, uint64_t* d_msg_end, void* d_ws, size_t ws_bytes,
                                 hipStream_t stream);

/* ------------------------------------------ PUT message serialization (write side, row a10) */

/* One PUT message to lay out (PutMessageFormatInputStream.java:76-124 / :133-162 for header V1):
 *   header (V1 34 B / V2 38 B / V3 40 B, MessageFormatRecord.java:467-486, :696-725, :951-981)
 *   store key (its serialized bytes, e.g. MockId: short length + id)
 *   [BlobEncryptionKey_Format_V1 record: version 1, int size, key, CRC]  (header V2/V3 only)
 *   BlobProperties_Format_V1 record: version 1, BlobPropertiesSerDe bytes, CRC
 *   UserMetadata_Format_V1 record: version 1, int size, metadata, CRC
 *   Blob_Format_V3 record: version 3, short blobType, byte isCompressed, long size, content, CRC
 * Every CRC is CRC-32 of its record (header: of its first size-8 bytes) stored as a big-endian
 * long with the upper 32 bits zero; all integers big-endian. 80 bytes, no padding. */
typedef struct ambrycrc_put_desc {
  uint64_t out_off;      /* message start in the output buffer */
  uint64_t key_src;      /* field offsets in the fields buffer (unused when fields == NULL) */
  uint64_t enckey_src;
  uint64_t props_src;
  uint64_t usermeta_src;
  uint64_t blob_src;     /* content offset in the blobs buffer (unused when blobs == NULL) */
  uint64_t blob_len;
  uint32_t key_len;
  int32_t enckey_len;    /* -1: no encryption-key record */
  uint32_t props_len;
  uint32_t usermeta_len;
  int16_t life_version;  /* header V3 */
  int16_t blob_type;
  uint8_t compressed;
  uint8_t header_version; /* 1, 2 or 3 (MessageFormatRecord.headerVersionToUse) */
  uint8_t reserved[2];
} ambrycrc_put_desc;

/* Where the variable fields of message d go, relative to its start: offsets[0..4] = key,
 * encryption key (0 when absent), blob-properties bytes, user-metadata bytes, blob content.
 * Returns the message length (header + key + records), or 0 for an invalid descriptor. A
 * caller that receives the fields straight into the output at these offsets (a Netty buffer
 * read into the log buffer) serializes in place: pass fields == NULL and blobs == NULL below. */
uint64_t ambrycrc_put_layout(const ambrycrc_put_desc* d, uint64_t* offsets);

/* One message on the CPU: header, key, records, every CRC trailer, at out + d->out_off
 * (out_cap bytes in out). crcs[5] (nullable) = header, encryption key (0 if absent), properties,
 * user metadata, blob record CRCs. The write side of MessageFormatInputStream.read*
 * (MessageFormatInputStream.java:40-96) for one PUT. */
int ambrycrc_serialize_put_host(const ambrycrc_put_desc* d, const uint8_t* fields, const uint8_t* blobs, uint8_t* out,
                                uint64_t out_cap, uint32_t* crcs);

/* m messages on the GPU (d_desc: device array): one thread per message writes the header and
 * record prefixes. With d_fields or d_blobs given, the batch CRC kernels read key / encryption
 * key / properties / user metadata (from d_fields) and blob contents (from d_blobs) once, write
 * them into place and CRC them in the same pass (copy-through); a last kernel extends those CRCs
 * over the record prefixes and writes the trailers. d_fields / d_blobs NULL: those bytes are
 * already in place in d_out (ambrycrc_put_layout) and are CRC'd there; both NULL is a single
 * read pass. d_msg_len[m] (nullable): message lengths. Descriptors must be valid
 * (ambrycrc_put_layout != 0), messages must not overlap, and the source buffers must not
 * overlap d_out.
 * Asynchronous on `stream`; d_ws >= ambrycrc_serialize_puts_workspace_bytes(m) or NULL. */
size_t ambrycrc_serialize_puts_workspace_bytes(size_t m);
int ambrycrc_serialize_puts_dev(const ambrycrc_put_desc* d_desc, size_t m, const uint8_t* d_fields,
                                const uint8_t* d_blobs, uint8_t* d_out, uint64_t* d_msg_len, void* d_ws,
                                size_t ws_bytes, hipStream_t stream);

/* Status bits ambrycrc_transform_messages_dev adds to the AMBRYCRC_MSG_* verify bits. */
#define AMBRYCRC_MSG_NOT_PUT (1u << 10)     /* an update record: "Message cannot be anything rather than put record" */
#define AMBRYCRC_MSG_NO_ROOM (1u << 12)     /* the re-serialized message did not fit in out_cap */
#define AMBRYCRC_MSG_NOT_ENCODABLE (1u << 13) /* a BlobProperties string holds a non-ASCII byte: the
                                               reference's V5 re-serialization overruns its buffer,
                                               whose size counts String.length() (BlobPropertiesSerDe
                                               .java:43-54 vs :83-103; PutMessageFormatInputStream.java
                                               :83-90), and the transform throws */

/* Replication's ValidatingTransformer.transform (ambry-messageformat/.../ValidatingTransformer.java:46-104)
 * for m stored messages at d_msg_off[i] in [d_region, d_region + region_len): every CRC is verified
 * (ambrycrc_verify_messages_dev), update records are refused, the fields are deserialized
 * (key, encryption key, properties, user metadata, blob content / type / compression), and every
 * clean PUT is re-serialized by PutMessageFormatInputStream's layout -- blob properties at
 * BlobPropertiesSerDe VERSION_5 (ValidatingTransformer.java:77,87-89; AMBRYCRC_MSG_NOT_ENCODABLE
 * when a property string is not ASCII), blob record at Blob_Format_V3 -- with header version
 * `header_version` (1, 2 or 3: MessageFormatRecord.headerVersionToUse; V1 drops the encryption key,
 * as createStreamWithMessageHeaderV1 does) and life version d_life_version[i], written as given,
 * negatives included (ValidatingTransformer.java:90; nullable: the stored header's, 0 for V1/V2)
 * -- all CRCs recomputed -- packed in message order into
 * [d_out, d_out + out_cap). Outputs (device arrays of m): d_status (AMBRYCRC_MSG_* bits, 0 =
 * transformed), d_out_len (0 when not transformed), d_out_off (nullable; the message's offset in
 * d_out). Bytes of d_out outside the returned spans are unspecified (a clean batch is copied while
 * it is verified; a batch with a failing message is then rebuilt). d_out must not overlap the
 * region. Enqueued on `stream`; d_ws >= ambrycrc_transform_workspace_bytes(m) or NULL. The
 * store-key comparison with the index entry stays with the caller (it owns the StoreKey type).
 * Fast path (header_version 3, region mode on, at most 40 KiB of region per message
 * (AMBRYCRC_XFORM_FAST_MAX at init overrides; 0 = never), workspace room for the region's run sums
 * -- the default workspace has it): one pass verifies the messages while copying the region into d_out
 * and rewrites the headers' life versions; it takes the batch when every message is a clean PUT
 * stored at header V3 with VERSION_5 properties and a Blob_Format_V3 record, back to back from
 * d_msg_off[0]; otherwise the general path redoes the batch, with the same outputs.
 * Asynchronous, as every *_dev entry: the fast path's verdict stays on the device and the general
 * path is enqueued behind it (each of its kernels returns at once when the fast path took the
 * batch), so the call never blocks and may be captured into a HIP graph (the workspace must then
 * be the caller's, or the stream's default one grown by an earlier uncaptured call). With
 * ambrycrc_set_transform_verdict(device, 1) an uncaptured call instead reads the verdict back --
 * one synchronization of `stream`, blocking the calling thread -- and enqueues the general path
 * only when it is needed (no empty dispatches); a capturing stream always gets the device form. */
size_t ambrycrc_transform_workspace_bytes(size_t m);

/* Output size contract of the transform. A transformed message is at most
 * AMBRYCRC_TRANSFORM_GROWTH_MAX bytes longer than the stored message it comes from:
 *   header V1 (34 B) -> V3 (40 B)                                   +6
 *   BlobProperties SerDe V1 -> VERSION_5 (account, container, encrypted, three null strings) +17
 *   Blob_Format_V1 head (10 B) -> Blob_Format_V3 head (13 B)          +3
 * (every other record keeps its size; a V1 output header drops the encryption-key record). The
 * reference sizes its buffer from the same fields: PutMessageFormatInputStream.java:88-90,122 and
 * BlobPropertiesSerDe.java:43-54, MessageInfo size at ValidatingTransformer.java:91.
 * ambrycrc_transform_out_bound(region_len, m) = region_len + m * AMBRYCRC_TRANSFORM_GROWTH_MAX
 * (saturating): an out_cap that never yields AMBRYCRC_MSG_NO_ROOM when no two messages share region
 * bytes (a log region, a GetResponse) -- the cap for ambrycrc_transform_messages_dev/_host and, with
 * m = 1 and the stored message's length, for ambrycrc_transform_message_cpu. */
#define AMBRYCRC_TRANSFORM_GROWTH_MAX 26
uint64_t ambrycrc_transform_out_bound(uint64_t region_len, size_t m);

int ambrycrc_transform_messages_dev(const uint8_t* d_region, uint64_t region_len, const uint64_t* d_msg_off, size_t m,
                                    const int16_t* d_life_version, int header_version, uint8_t* d_out,
                                    uint64_t out_cap, uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_status,
                                    void* d_ws, size_t ws_bytes, hipStream_t stream);

/* ------------------------------------- CRC-trailered records (store files, headers) */

/* Item i = [off[i], off[i] + len[i]) ends in the big-endian 8-B CRC (a long, high word zero)
 * of its first len[i] - 8 bytes. d_mismatch[i] = 1 iff the stored long differs from the
 * computed CRC, or len[i] < 8 (where the reference throws). *d_mismatch_count (caller zeroes
 * it) counts them. Either output may be NULL. Batch form of
 * IndexSegment.checkDataIntegrityInByteBufferWithCRC (ambry-store/.../IndexSegment.java:727-735,
 * every index segment file at store start-up), the LogSegment header check
 * (LogSegment.java:130-140) and the user-metadata CRC of RestUtils.java:813-814. */
size_t ambrycrc_trailed_workspace_bytes(size_t n);
int ambrycrc_verify_trailed_dev(const uint8_t* d_base, const uint64_t* d_off, const uint64_t* d_len,
                                uint8_t* d_mismatch, uint32_t* d_mismatch_count, size_t n, void* d_ws,
                                size_t ws_bytes, hipStream_t stream);

/* The same for n host buffers (whole files read or mapped from disk): mismatch[n] host array.
 * The bodies go through ambrycrc_batch_host; synchronous. */
int ambrycrc_verify_trailed_host(const void* const* ptrs, const uint64_t* lens, uint8_t* mismatch, size_t n,
                                 int device, int pinned);

/* ambrycrc_verify_messages_dev for a region in HOST memory (a log segment read or mapped
 * from disk: BlobStoreRecovery's scan, a GET of stored messages). Messages are staged in
 * offset order through the context's pinned slabs (64 MiB, up to 65,536 messages each; a
 * message larger than a slab gets its own staging buffer), each slab holding the span its
 * messages cover, so the status bits and message ends equal those of the whole region.
 * pinned != 0: region is hipHostMalloc'd / registered (copied by DMA directly). status[m],
 * msg_end[m] (may be NULL): host arrays. Synchronous. */
int ambrycrc_verify_messages_host(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                                  uint32_t* status, uint64_t* msg_end, int device, int pinned);

/* ambrycrc_transform_messages_dev for a region in HOST memory (replication's batch: the messages of
 * one GetResponse, MessageSievingInputStream.java:130,278-288 over ReplicaThread.java:1810-1815).
 * Messages are staged in index order through the context's pinned slabs (runs of consecutive
 * messages whose span fits 64 MiB; a message larger than a slab gets its own buffers) and each
 * slab's re-serialized messages come back through pinned memory. Outputs equal those of one
 * ambrycrc_transform_messages_dev call over the whole region: out[0 .. out_cap) packed in message
 * order, out_off[i] (nullable; UINT64_MAX when not transformed), out_len[i], status[i] (host arrays);
 * life_version (nullable) host int16[m], written as given on either leg. out_cap = ambrycrc_transform_out_bound(region_len, m)
 * never yields AMBRYCRC_MSG_NO_ROOM for messages that share no bytes. pinned != 0: region is
 * hipHostMalloc'd / registered. Synchronous. */
int ambrycrc_transform_messages_host(const uint8_t* region, uint64_t region_len, const uint64_t* msg_off, size_t m,
                                     const int16_t* life_version, int header_version, uint8_t* out, uint64_t out_cap,
                                     uint64_t* out_off, uint64_t* out_len, uint32_t* status, int device, int pinned);

/* Host-side message chain for a log region in host memory (the sequential hop of
 * BlobStoreRecovery.recover, BlobStoreRecovery.java:43-110): starting at `start`,
 * read each header (V1/V2/V3, header CRC checked) and follow its size to the next
 * message; stops at the first unparseable header or region end. Writes up to
 * `max` message offsets to offs; returns the count. */
size_t ambrycrc_chain_messages_host(const uint8_t* region, uint64_t region_len, uint64_t start, uint64_t* offs,
                                    size_t max);

/* One message on the CPU, for per-message callers (a GET of one blob through
 * MessageFormatSend.java:131-139, BlobStoreRecovery's per-message read): the checks of
 * ambrycrc_verify_messages_dev (header, every record CRC, record versions and size fields) for
 * the message at region + off, with the CLMUL host loop. *status = AMBRYCRC_MSG_* bits;
 * *msg_end (nullable) = offset one past the message, or 0 when unparseable. */
int ambrycrc_verify_message_cpu(const uint8_t* region, uint64_t region_len, uint64_t off, uint32_t* status,
                                uint64_t* msg_end);

/* ValidatingTransformer.transform (ValidatingTransformer.java:46-104) for one stored message on
 * the CPU, as ambrycrc_transform_messages_dev does it for a batch: verify, refuse update records,
 * deserialize, re-serialize at header_version (1..3) with life_version (< 0: the stored one;
 * V1/V2 headers carry none) into out[0 .. *out_len); the blob properties are re-encoded at
 * BlobPropertiesSerDe VERSION_5 whatever version they were stored at. *status = AMBRYCRC_MSG_*
 * verify bits | AMBRYCRC_MSG_NOT_PUT / _BAD_RECORD / _NOT_ENCODABLE / _NO_ROOM (out_cap too
 * small; *out_len 0); 0 = transformed.
 * out must not overlap the region. */
int ambrycrc_transform_message_cpu(const uint8_t* region, uint64_t region_len, uint64_t off, int life_version,
                                   int header_version, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                                   uint32_t* status);

/* ------------------------------------------------------- host-resident batch */

/* CRC-32 of n host chunks (ptrs[i], lens[i]) on `device`: chunks are packed into
 * pinned staging buffers, copied with hipMemcpyAsync on two streams
 * (double-buffered, copy of slab k+1 overlapping the kernels of slab k) and
 * CRC'd in HBM. Synchronous. Inputs that already live in pinned memory
 * (hipHostMalloc / hipHostRegister'd Netty arenas) are copied without a
 * host-side memcpy when `pinned` is nonzero.
 * This is the PUT path's entry: the bytes start in a Netty ByteBuf
 * (ambry-network/.../NettyServerRequest.java:35,54) or a FileChannel prefetch
 * (ambry-store/.../StoreMessageReadSet.java:170-188). */
int ambrycrc_batch_host(const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in, uint32_t* out,
                        size_t n, int device, int pinned);

/* Host-resident dispatch of the *_host entries (ambrycrc_batch_host, _verify_messages_host,
 * _transform_messages_host, and through them _verify_trailed_host and _range_checksums_host;
 * ambrycrc_batch_multi decides once for its whole batch). Bytes that live in pageable host memory
 * reach the GPU over PCIe (~51 GiB/s per GPU) while the CPU's CLMUL loop hashes them
 * at ~9 GiB/s per thread: policy 0 (auto, the default) takes the CPU leg -- the same outputs, on
 * ambrycrc_host_rates' CPU threads -- when their rate beats the GPU host path's, and the GPU for
 * pinned bytes (pinned != 0: the caller registered them for DMA); 1 = always the GPU; 2 = always
 * the CPU. device < 0 in those entries means the CPU leg (no context needed). Returns the previous
 * policy. Replaces nothing in the reference, whose callers (NettyServerRequest.java:35,54,
 * StoreMessageReadSet.java:170-188) hold exactly such host buffers. */
int ambrycrc_set_host_policy(int device, int policy);
/* The rates the auto policy compares for ambrycrc_batch_host: *cpu_gibps (the CLMUL CPU leg's rate
 * at the device's thread budget: as its pageable calls of >= 64 MiB measured it, else the calibration
 * at that budget -- each thread over its own slice of a buffer past the L3), *gpu_gibps (the GPU host
 * path: 51 GiB/s measured, refreshed by each pageable GPU call of >= 64 MiB; under auto every 16th
 * such call takes the other leg, so both stay current), *cpu_threads (the budget,
 * ambrycrc_set_host_cpu_threads). Returns the leg auto takes for pageable bytes (0 CPU, 1 GPU), or
 * < 0. Any output may be NULL. device -1: the process's budget and CPU rate, no GPU (gpu 0). */
int ambrycrc_host_rates(int device, double* cpu_gibps, double* gpu_gibps, int* cpu_threads);
/* The CPU budget of the host-resident CPU leg: how many threads ambrycrc_batch_host,
 * _verify_messages_host and _transform_messages_host use on `device` when they take it, and the budget
 * at which auto rates that leg. threads 0 = the default: the process's budget (this call with device
 * -1), else AMBRYCRC_CPU_THREADS, else half the CPUs this process may use (affinity, cgroup v2 quota,
 * OMP_NUM_THREADS) -- the other half stays with the server's own network and disk threads, which the
 * reference runs on the same cores (NettyServerRequest.java:35,54, StoreMessageReadSet.java:170-188).
 * Returns the previous setting (0 = default), AMBRYCRC_EINVAL (threads outside 0..256) or
 * AMBRYCRC_ENOINIT. The CRC batch's measured CPU rates are kept per budget; a change forgets the message
 * legs' (they were at the old budget). */
int ambrycrc_set_host_cpu_threads(int device, int threads);
/* Runs the CPU leg's calibration at `device`'s budget now (once per thread count per process; up to
 * 256 MiB written and hashed by the budget's threads, ~50-200 ms) instead of inside the first auto
 * decision that needs it, and returns the rate in *cpu_gibps (may be NULL). device -1: the process's
 * budget. A server calls it at start-up, before traffic. */
int ambrycrc_host_calibrate(int device, double* cpu_gibps);
/* The leg the device's last host call took: 0 CPU, 1 GPU, -1 none yet. */
int ambrycrc_last_host_path(int device);
/* The rates auto compares for the host message entries (op 0: ambrycrc_verify_messages_host, 1:
 * ambrycrc_transform_messages_host), GiB/s of region bytes: each leg's rate as its calls of >= 64 MiB
 * measured it (an EWMA; the CPU leg starts at a share of the CRC rate, the GPU leg at round 5's
 * measurement); under auto every 16th such pageable call takes the other leg to refresh it.
 * Returns the leg auto takes for pageable bytes (0 CPU, 1 GPU), or < 0. */
int ambrycrc_host_msg_rates(int device, int op, double* cpu_gibps, double* gpu_gibps);

/* ambrycrc_batch_host across several GPUs of this process: the n
 * chunks are split into ndev contiguous ranges by ambrycrc_shard_by_bytes, range g runs ambrycrc_batch_host on devices[g]
 * from its own host thread, and the calls are joined. devices == NULL means
 * 0..ndev-1; a device may appear more than once (its ranges then run one after the
 * other). Every listed device must have been ambrycrc_init'ed. Returns the first
 * nonzero status of any range; out[] is complete only on AMBRYCRC_OK.
 * This is the single-JVM form of the per-GPU sharding the bench runs as one
 * process per GPU: a storage node scanning many partitions in one process. */
int ambrycrc_batch_multi(const void* const* ptrs, const uint64_t* lens, const uint32_t* crc_in, uint32_t* out,
                         size_t n, const int* devices, int ndev, int pinned);

/* ------------------------------------- multi-GPU batch + RCCL all-gather */

/* Shards of a batch: chunk ranges [cuts[g], cuts[g+1]) of about equal BYTES (mixed sizes are
 * balanced by bytes, not by count): shard g takes the chunks whose start byte s (prefix sum of
 * lens) satisfies g/nshards <= s/total < (g+1)/nshards; an all-empty batch is split by count.
 * cuts[nshards + 1]. Host arithmetic, no device. */
int ambrycrc_shard_by_bytes(const uint64_t* lens, size_t n, int nshards, size_t* cuts);

/* An RCCL communicator over the GPUs that share one batch (opaque). RCCL (librccl.so.1) is
 * loaded on first use; without it these calls return AMBRYCRC_ECOMM. */
typedef struct ambrycrc_comm ambrycrc_comm;
#define AMBRYCRC_UNIQUE_ID_BYTES 128

/* One process driving ndev GPUs (devices == NULL: 0..ndev-1; no device twice). Every device
 * must also be ambrycrc_init'ed before a batch runs on it. */
int ambrycrc_comm_init_all(const int* devices, int ndev, ambrycrc_comm** comm);
/* One process per GPU: rank 0 calls ambrycrc_unique_id and sends the 128 bytes to every rank
 * (any channel); each rank then calls ambrycrc_comm_init_rank for its own device. */
int ambrycrc_unique_id(uint8_t* id);
int ambrycrc_comm_init_rank(const uint8_t* id, int nranks, int rank, int device, ambrycrc_comm** comm);
/* Waits for the communicator's devices to go idle, then releases it. */
int ambrycrc_comm_destroy(ambrycrc_comm* comm);
int ambrycrc_comm_size(const ambrycrc_comm* comm);

/* One GPU's part of a multi-GPU batch. */
typedef struct ambrycrc_shard {
  int device;
  const uint8_t* d_base;    /* the shard's chunks: d_base + d_off[i], d_len[i] bytes (device arrays) */
  const uint64_t* d_off;
  const uint64_t* d_len;
  const uint32_t* d_crc_in; /* nullable */
  size_t n;                 /* chunks in this shard */
  uint32_t* d_gathered;     /* on `device`: the CRCs of EVERY shard, shard order (sum of all n words) */
  hipStream_t stream;       /* work is enqueued here (NULL: the device's null stream) */
} ambrycrc_shard;

/* Single process: shards[g] runs on comm's g-th device (shards[g].device must match); each
 * shard's CRCs are computed on its GPU (ambrycrc_batch_dev), then one ncclAllGather of the
 * uint32 CRCs over xGMI leaves the whole batch's CRCs in every shard's d_gathered.
 * Asynchronous: enqueued on the shards' streams. The batch callers are replication verify
 * (ambry-replication/.../ReplicaThread.java:1810-1815) and the recovery scan of a log
 * (ambry-store/.../BlobStoreRecovery.java:43-110), run for many partitions in one server. */
int ambrycrc_batch_dev_multi(ambrycrc_comm* comm, const ambrycrc_shard* shards, int nshards);

/* One process per GPU: this rank's shard (`mine`, on the communicator's device) and the shard
 * sizes of all ranks (counts[nranks], identical on every rank; counts[rank] == mine->n). Every
 * rank must call it for the gather to complete. Asynchronous, as above. */
int ambrycrc_batch_dev_gather(ambrycrc_comm* comm, const ambrycrc_shard* mine, const uint64_t* counts);

/* The all-gather layout both entries above use, for shard sizes counts[nranks]: every rank sends
 * a segment of *width CRCs (the largest count rounded up to 64); rank r's CRCs sit at
 * [r * width, r * width + counts[r]) of the nranks * width gather buffer. *in_place (every count
 * == width, width > 0): that buffer is d_gathered itself; otherwise a padded scratch buffer,
 * whose segments are then copied to d_gathered[starts[r] .. starts[r + 1]) (starts[nranks + 1],
 * prefix sums of counts). Any output pointer may be NULL. Host arithmetic, no device. */
int ambrycrc_gather_layout(const uint64_t* counts, int nranks, uint64_t* width, int* in_place, uint64_t* starts);

/* The compaction step of that layout on host memory: out[starts[r] ..] = padded[r * width ..]
 * for every rank (the same copy list the device path enqueues; a gloo / host-side gather of the
 * padded segments finishes here). padded holds nranks * width words, out sum(counts). */
int ambrycrc_gather_compact_host(const uint32_t* padded, const uint64_t* counts, int nranks, uint32_t* out);

/* One-pass PUT CRCs (§8f row 2). For each of n PUT requests whose blob CRC blob_crc[i]
 * (over blob_len[i] bytes, e.g. from ambrycrc_batch_dev/ambrycrc_batch_host) is known:
 *   wire_out[i]   = crc32(fields[i] || blob)   -- PutRequest.prepareBuffer's CRC over blobId,
 *                   properties, user metadata, blobType, key, isCompressed, blobSize and the blob
 *                   (ambry-protocol/.../PutRequest.java:238-283), verified by PutRequest_V5.readFrom
 *                   (:497-521)
 *   record_out[i] = crc32(prefix[i] || blob)   -- the Blob_Format_V3 record CRC seeded by its 13-B
 *                   prefix (MessageFormatRecord.java:1789-1795, PutMessageFormatInputStream.java:116-120)
 * so the blob bytes are scanned once instead of twice (three times counting the receive check).
 * fields/prefix are host byte arrays; either output may be NULL. Host-only arithmetic. */
int ambrycrc_put_crcs(const uint8_t* const* fields, const uint64_t* field_len, const uint8_t* const* prefix,
                      const uint64_t* prefix_len, const uint32_t* blob_crc, const uint64_t* blob_len, size_t n,
                      uint32_t* wire_out, uint32_t* record_out);

/* CRC-32 of byte ranges of one file image in host memory, on `device` (§8f row 3).
 * Replaces FileStore.getChecksumsForRanges (ambry-store/.../FileStore.java:567-595)
 * with its exact semantics: range i covers [first[i], second[i]) -- `second - first`
 * bytes, as the reference computes `size` (StoreFileCopyHandler.getChecksumRanges
 * builds second = start + size - 1, so the last byte of each range is not covered) --
 * truncated at EOF like the reference's FileChannel.read, empty past EOF. Returns
 * AMBRYCRC_EINVAL, computing nothing, if any range has first < 0, second < 0 or
 * first > second (the reference's IllegalArgumentException). out[i] is the value
 * the reference renders with Long.toString. */
int ambrycrc_range_checksums_host(const uint8_t* file, uint64_t file_len, const int64_t* first, const int64_t* second,
                                  size_t n, uint32_t* out, int device);

/* =====================================================================================
 * DIAGNOSTICS -- for benchmarks, profiles and tests, not for production callers. Nothing in
 * the reference corresponds to these entries. Every production path above is correct and
 * tuned with their defaults; they select kernel shapes for A/B runs (set_variant, set_grid,
 * set_window, set_region_mode, set_transform_verdict), time kernels (timing_*), report which
 * form a call took (last_message_mode, last_transform_path), fill synthetic data
 * (fill_random_dev), probe bandwidth (debug_readbw_dev) and expose the table image to the CPU
 * kernel model (debug_table_image). The JNI shim binds none of them.
 * ===================================================================================== */

/* ------------------------------------------------------- tuning / telemetry */

/* Kernel variant (0..29; crc32_kernels.h lists them). 0..13: sweep-kernel shapes (blocks in
 * flight per lane, load policy, prefetch scheme, lane runs) for every chunk; 14..19: sweep
 * variant 0 plus a separate group kernel for whole chunks up to 2..16 KiB; 20..26: the
 * group phase fused into the sweep launch. Group modes engage for batches of >= 16384
 * chunks; smaller batches take the sweep for every chunk (latency).
 * 28 = 64-B lane runs (coalesced loads, quad transpose by v_cndmask_b32_dpp, one
 * fold per 64 B) with the group phase for whole chunks <= 16 KiB sized per size class
 * (4 / 8 / 16 lanes per chunk, 64-B lane runs in the 8- and 16-lane groups) and spread over
 * all waves per class. Default 29 = 28 with the wave's priority raised (s_setprio 3)
 * while it issues each super-block's loads.
 * 100..102 are timing diagnostics that produce wrong CRCs. ambrycrc_get_variant returns
 * the current one. */
int ambrycrc_set_variant(int device, int variant);
int ambrycrc_get_variant(int device);
/* Message verify (ambrycrc_verify_messages_dev / _host) of a region of at most 6 KiB per
 * message: region mode sweeps the region once as contiguous memory, keeping the raw CRC of every
 * 64-B run, and assembles each record's CRC from the runs it covers, re-reading only the two runs
 * its ends cut. 2 (the default): two passes -- the sweep, then one thread per message;
 * 1: one pass -- each CU's processor waves take the messages of its share of the region while its
 * streaming waves are still sweeping it (measured 1.5-14 % slower than 2 for verify: the
 * processors' dependent loads wait behind the saturated stream; it is the transform's fast path,
 * which runs when the mode is 1 or 2); 0: every record as a CRC job through the batch engine
 * (plan, group phase, sweep). AMBRYCRC_REGION=0 / 1 in the environment at init selects 0 / 1.
 * Same status bits every way.
 * ambrycrc_last_message_mode: the form the device's last message verify took (0 / 1 / 2; -1
 * before the first), for profiles that must say which kernels they timed. */
int ambrycrc_set_region_mode(int device, int enable);
int ambrycrc_get_region_mode(int device);
int ambrycrc_last_message_mode(int device);
/* Diagnostic, for tests and profiles only: the path the device's last ambrycrc_transform_messages_dev
 * call (or _host slab) took: 1 = the one-pass fast path alone (header V3, every message a clean dense V3
 * PUT with canonical properties), 0 = the general path (after the fast pass gave up, or without it),
 * -1 = none yet. One word per device, written by every transform on every stream: with concurrent
 * transforms it names whichever finished last. When that call left the verdict on the device (the
 * default), this waits for the whole device to go idle (hipDeviceSynchronize) and reads it -- do not
 * call it while another thread captures a graph. */
int ambrycrc_last_transform_path(int device);
/* How ambrycrc_transform_messages_dev learns whether its fast path took the batch: 0 (the default;
 * AMBRYCRC_XFORM_HOST_VERDICT=1 at init sets 1) = on the device, the general path enqueued behind a
 * device gate -- asynchronous; 1 = read back by the calling thread (one stream synchronization per
 * call, 256 calls in flight at most; more take the device form). Returns the previous value. */
int ambrycrc_set_transform_verdict(int device, int host);
/* Serialize copy mode (ambrycrc_serialize_puts_dev with both source buffers) streams messages of at most
 * `bytes` bytes (put_stream_kernel + put_stream_seal_kernel; at most 6144, the
 * default); 0 sends every message through the job path. Returns the previous value, or < 0. For A/B runs
 * and tests: both forms write the same bytes. */
long ambrycrc_set_put_stream_max(int device, long bytes);
/* Grid size of the persistent sweep kernel (workgroups; 0 = one per CU). */
int ambrycrc_set_grid(int device, int workgroups);

/* Sweep rounds: a batch of more than `bytes` is swept in rounds of at most that many bytes,
 * so the waves read inside one window at a time (default 32 GiB; 0 = one round over the
 * whole batch; otherwise >= 1 MiB). Same results either way. */
int ambrycrc_set_window(int device, uint64_t bytes);

/* When enabled, every batch's CRC kernels (group kernel + sweep kernel, not the plan) are
 * bracketed by HIP events on the caller's stream; ambrycrc_timing_collect() waits for them
 * and returns the sum and count of those durations since the last collect. */
int ambrycrc_timing_enable(int device, int enable);
int ambrycrc_timing_collect(int device, double* total_ms, int* launches);
/* As ambrycrc_timing_collect, but writes each launch's duration (ms, launch order) to
 * ms_out[0 .. min(cap, launches)) so a caller can report the median; *launches is the total. */
int ambrycrc_timing_collect_each(int device, float* ms_out, int cap, int* launches);

/* Number of workgroups the sweep kernel launches with on `device` (0 if unknown). */
int ambrycrc_grid_size(int device);

/* ------------------------------------------------------- synthetic data and probes (diagnostics) */

/* Fill d_dst with the deterministic splitmix64 byte stream (byte i = byte i&7 of
 * splitmix64_mix(seed + ((stream_off+i)/8 + 1) * 0x9E3779B97F4A7C15)).
 * d_dst must be 16-B aligned and stream_off a multiple of 16. For benchmarks. */
int ambrycrc_fill_random_dev(uint8_t* d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream_off,
                             hipStream_t stream);

/* Read-bandwidth probe (no CRC arithmetic) over [d_base, d_base+nbytes) with the
 * sweep kernel's grid and access pattern (variant 0: 256 KiB tiles; 1 = the same with
 * nontemporal loads; 2 = plain grid-stride stream; 3 = contiguous per-wave shares, NT;
 * 4 = shares entered at a per-wave rotation, NT; 16 + k = the group phase's shape for chunks of 1 KiB << k,
 * 16-lane groups, 4 chunks per wave round, one 1 KiB super-block per group prefetched). d_out needs grid*1024
 * words. Measures the achievable HBM read roof the CRC kernels are compared against.
 * Copy probes (they WRITE the buffer's upper half): 32 + k = the group shape above reading
 * [0, nbytes/2 - 4096) and storing each piece at the same offset from d_base + nbytes/2;
 * 40 + k = the same with the destination 11 B further (unaligned stores); 48 = contiguous
 * per-wave shares; 49 / 50 = grid-stride copy over 32 blocks of 256 threads per CU, plain /
 * nontemporal stores (the plain copy roof).
 * FETCH_SIZE calibration (60 / 61 / 62): every 128-B line of the largest power-of-two number of
 * lines in nbytes read once, in scattered order, by one 16-B / 4-B / unaligned 8-B load. */
int ambrycrc_debug_readbw_dev(const uint8_t* d_base, uint64_t nbytes, uint32_t* d_out, int variant,
                              hipStream_t stream);

/* Copy of the table image (the LDS image kLdsBytes, 64 words x^(8*2^k), the nibble sets of
 * x^(-8*2^k), k = 0..5, then region pass 2's words -- head-run initial registers, byte masks, the
 * x^(8*256) byte tables and the un-shift sets: kImgBytes in all) into host memory `out` (for
 * tests that model the kernel on the CPU). Returns the byte size, or <0. */
long ambrycrc_debug_table_image(uint32_t* out, size_t max_words);

#ifdef __cplusplus
}
#endif
#endif /* AMBRYCRC_H */
