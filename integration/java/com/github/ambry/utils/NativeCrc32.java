/*
 * NativeCrc32 -- drop-in java.util.zip.Checksum backed by libambrycrc (MI355X / gfx950 CRC-32
 * engine), for ambry-utils. Bit-exact with com.github.ambry.utils.Crc32 and java.util.zip.CRC32
 * (CRC-32/ISO-HDLC).
 *
 * Binding: libambrycrc_jni.so (ambry_amd/jni/ambrycrc_jni.c), which links libambrycrc.so and
 * libambrycrc_jnicore.so. Native failures are thrown by the shim as exceptions
 * (IndexOutOfBoundsException, IllegalArgumentException, NullPointerException,
 * OutOfMemoryError, IllegalStateException); a CRC value is never a status code.
 *
 * Replaces: Crc32 (ambry-utils/.../utils/Crc32.java:34-149), and -- with
 * ambry-utils-checksum-retype.patch applied -- the CRC32 instances of CrcInputStream
 * (CrcInputStream.java:28,40) and CrcOutputStream (CrcOutputStream.java:25,36).
 */
package com.github.ambry.utils;

import java.nio.ByteBuffer;
import java.util.zip.Checksum;


public final class NativeCrc32 implements Checksum {
  /** Whether libambrycrc_jni loaded. Crc32 consults it, so a JVM without the library keeps the pure-Java loop. */
  private static final boolean LOADED = load();

  /**
   * com.github.ambry.utils.Crc32 runs updates of at least this many bytes through the library
   * (ambry-utils-crc32-native.patch); Integer.MAX_VALUE when the library did not load or
   * -Dambry.crc32.native=false. Below it the JNI crossing costs more than the Java slice-by-8
   * loop (-Dambry.crc32.native.min.bytes, default 256).
   */
  static final int CRC32_MIN_BYTES = crc32MinBytes();

  private static boolean load() {
    try {
      System.loadLibrary("ambrycrc_jni");
      return true;
    } catch (UnsatisfiedLinkError | SecurityException e) {
      return false;
    }
  }

  private static int crc32MinBytes() {
    if (!LOADED || "false".equals(System.getProperty("ambry.crc32.native"))) {
      return Integer.MAX_VALUE;
    }
    return Math.max(1, Integer.getInteger("ambry.crc32.native.min.bytes", 256));
  }

  /** True when libambrycrc_jni loaded; every other method throws UnsatisfiedLinkError otherwise. */
  public static boolean isAvailable() {
    return LOADED;
  }

  /** Finalized value (zlib convention, starts at 0); Crc32.java keeps the inverted register. */
  private int crc;

  /** Crc32.update(int), Crc32.java:146-148: the low 8 bits of b. */
  @Override
  public void update(int b) {
    crc = nativeUpdateByte(crc, b);
  }

  /** Crc32.update(byte[], int, int), Crc32.java:55-98. Bounds as java.util.zip.CRC32. */
  @Override
  public void update(byte[] b, int off, int len) {
    if (b == null) {
      throw new NullPointerException();
    }
    if (off < 0 || len < 0 || off > b.length - len) {
      throw new ArrayIndexOutOfBoundsException();
    }
    crc = nativeUpdateArray(crc, b, off, len);
  }

  /** Crc32.update(ByteBuffer), Crc32.java:100-143: consumes position..limit. */
  @Override
  public void update(ByteBuffer buffer) {
    crc = updateBuffer(crc, buffer);
  }

  /**
   * The finalized CRC `crc` continued over buffer's position..limit, which it consumes (Crc32.java:100-143).
   * Crc32 calls it with its register inverted.
   */
  static int updateBuffer(int crc, ByteBuffer buffer) {
    int pos = buffer.position();
    int len = buffer.remaining();
    if (len == 0) {
      return crc;
    }
    if (buffer.isDirect()) {
      crc = nativeUpdateDirect(crc, buffer, pos, len);
    } else if (buffer.hasArray()) {
      crc = nativeUpdateArray(crc, buffer.array(), buffer.arrayOffset() + pos, len);
    } else {  // read-only heap buffer: copy out
      byte[] tmp = new byte[len];
      buffer.duplicate().get(tmp);
      crc = nativeUpdateArray(crc, tmp, 0, len);
    }
    buffer.position(buffer.limit());
    return crc;
  }

  /** The finalized CRC `crc` continued over b[off, off + len); Crc32 checks the bounds first. */
  static int updateArray(int crc, byte[] b, int off, int len) {
    return nativeUpdateArray(crc, b, off, len);
  }

  /** update(ByteBuffer) over a gather list, e.g. PutChunk.verifyCRC's nioBuffers() (PutOperation.java:2041-2043). */
  public void updateAll(ByteBuffer[] buffers) {
    boolean allDirect = true;
    for (ByteBuffer b : buffers) {
      allDirect &= b.isDirect();
    }
    if (!allDirect) {
      for (ByteBuffer b : buffers) {
        update(b);
      }
      return;
    }
    crc = nativeUpdateDirectAll(crc, buffers);  // one JNI crossing
    for (ByteBuffer b : buffers) {
      b.position(b.limit());
    }
  }

  /** Crc32.getValue(), Crc32.java:44-47. */
  @Override
  public long getValue() {
    return crc & 0xffffffffL;
  }

  /** Crc32.reset(), Crc32.java:49-52. */
  @Override
  public void reset() {
    crc = 0;
  }

  /** CRC of A||B from crc(A), crc(B) and |B| (zlib crc32_combine). */
  public static long combine(long crc1, long crc2, long len2) {
    return nativeCombine((int) crc1, (int) crc2, len2) & 0xffffffffL;
  }

  /** Create the device context of GPU `device` (ambrycrc_init). Idempotent. */
  public static void init(int device) {
    nativeInit(device);
  }

  /**
   * CRCs of many direct-buffer chunks on GPU `device` (ambrycrc_batch_host: pinned staging, PCIe
   * copy, gfx950 kernels): out[i] = crc32(crcIn == null ? 0 : crcIn[i], bufs[i][pos[i], pos[i] + len[i])).
   */
  public static void batch(ByteBuffer[] bufs, int[] pos, int[] len, int[] crcIn, int[] out, int device) {
    // device < 0: the CPU leg; otherwise the library's host-resident dispatch (ambrycrc_set_host_policy)
    nativeBatchDirect(bufs, pos, len, crcIn, out, device);
  }

  /**
   * Verify every CRC of the messages at `offsets` in a log-segment region held in a direct buffer
   * (BlobStoreRecovery scan, GET, replication): status[i] = 0 when every CRC matches, else
   * AMBRYCRC_MSG_* bits (the lowest set bit is the record deserializeBlobAll would throw on);
   * ends[i] (may be null) = end offset of message i, 0 when its layout is invalid.
   */
  public static void verifyMessages(ByteBuffer region, long[] offsets, int[] status, long[] ends, int device) {
    // device < 0: the library's CPU leg; otherwise its host-resident dispatch picks the CPU threads or
    // GPU `device` for these (pageable) bytes, whichever hashes them faster (ambrycrc_set_host_policy)
    nativeVerifyMessages(region, offsets, status, ends, device);
  }

  /**
   * BlobStoreRecovery's hop from message to message (BlobStoreRecovery.java:43-110) over a log span in a
   * direct buffer (ambrycrc_chain_messages_host): from `start`, each header is read (version, header CRC,
   * sizes) and its message length followed; offsets[0 .. returned) get the message starts. The chain stops
   * at the first header that does not parse, at a message that runs past the buffer, or when `offsets` is
   * full. CPU only.
   */
  public static int chainMessages(ByteBuffer region, long start, long[] offsets) {
    return nativeChainMessages(region, start, offsets);
  }

  /**
   * One message on the CPU (ambrycrc_verify_message_cpu): deserializeBlobAll's checks (header, record
   * versions and sizes, every CRC) for the message at `offset` in a direct buffer. Returns the
   * AMBRYCRC_MSG_* bits (0: intact); end[0] (if end is non-null) = the message's end offset, 0 when
   * its layout is invalid.
   */
  public static int verifyMessage(ByteBuffer region, long offset, long[] end) {
    return nativeVerifyMessage(region, offset, end);
  }

  /**
   * ValidatingTransformer.transform for one stored message on the CPU (ambrycrc_transform_message_cpu):
   * verify, refuse update records, re-serialize at `headerVersion` (1..3) with `lifeVersion` (< 0:
   * the stored one) into `out` from position 0. Returns the status bits (0: transformed; MSG_NOT_PUT,
   * MSG_BAD_RECORD, MSG_NOT_ENCODABLE, MSG_NO_ROOM or verify bits otherwise); outLen[0] = bytes
   * written. An `out` of transformOutBound(storedSize, 1) bytes never yields MSG_NO_ROOM.
   */
  public static int transformMessage(ByteBuffer region, long offset, int lifeVersion, int headerVersion,
      ByteBuffer out, long[] outLen) {
    return nativeTransformMessage(region, offset, lifeVersion, headerVersion, out, outLen);
  }

  /**
   * ValidatingTransformer.transform for a batch of stored messages on GPU `device`
   * (ambrycrc_transform_messages_host): the messages at `offsets` in the direct buffer `region` (one
   * GetResponse's bytes, MessageSievingInputStream.java:130,278-288), re-serialized at `headerVersion`
   * with lifeVersions[i] (null: the stored ones) and packed in message order into the direct buffer
   * `out` from 0 -- its capacity is the output cap; transformOutBound(regionBytes, offsets.length)
   * never yields MSG_NO_ROOM. outOffsets[i] (may be null; -1 when not transformed), outLens[i] and
   * status[i] get each message's result.
   */
  public static void transformMessages(ByteBuffer region, long[] offsets, short[] lifeVersions, int headerVersion,
      ByteBuffer out, long[] outOffsets, long[] outLens, int[] status, int device) {
    // device < 0: the CPU leg; otherwise the library's host-resident dispatch (ambrycrc_set_host_policy)
    nativeTransformMessages(region, offsets, lifeVersions, headerVersion, out, outOffsets, outLens, status, device);
  }

  /**
   * Largest growth of one message under the transform (AMBRYCRC_TRANSFORM_GROWTH_MAX): header V1 to V3
   * (+6), BlobProperties SerDe V1 to VERSION_5 (+17), Blob_Format_V1 to V3 head (+3); the reference
   * sizes its output from the same fields (PutMessageFormatInputStream.java:88-90,122).
   */
  public static final int TRANSFORM_GROWTH_MAX = 26;

  /** Output capacity for m messages that share no bytes of a regionBytes-long region (ambrycrc_transform_out_bound). */
  public static long transformOutBound(long regionBytes, int m) {
    return regionBytes + (long) m * TRANSFORM_GROWTH_MAX;
  }

  /**
   * One-pass PUT CRCs (ambrycrc_put_crcs, SURVEY.md §8f row 2) for n = blobCrc.length PUTs whose blob CRC
   * blobCrc[i] over blobLen[i] bytes is already known (the router's chunk CRC, a batch call's output):
   * wireOut[i] = CRC of fields[i] followed by the blob -- PutRequest.prepareBuffer's wire CRC over the
   * serialized blobId ... blobSize fields and the blob (PutRequest.java:238-283) -- and recordOut[i] = CRC of
   * prefixes[i] followed by the blob -- the Blob_Format_V3 record CRC seeded by its 13-B prefix
   * (MessageFormatRecord.java:1789-1795, PutMessageFormatInputStream.java:116-120). Each field / prefix
   * buffer's position..limit is used and left unconsumed; heap buffers are copied out. Either output (with
   * its input list) may be null. No blob byte is read: both CRCs come from blobCrc by GF(2) combine.
   */
  public static void putCrcs(ByteBuffer[] fields, ByteBuffer[] prefixes, int[] blobCrc, long[] blobLen,
      int[] wireOut, int[] recordOut) {
    nativePutCrcs(directOrCopy(fields), directOrCopy(prefixes), blobCrc, blobLen, wireOut, recordOut);
  }

  /** The list with every heap buffer replaced by a direct copy of its position..limit (same position). */
  private static ByteBuffer[] directOrCopy(ByteBuffer[] bufs) {
    if (bufs == null) {
      return null;
    }
    ByteBuffer[] out = bufs;
    for (int i = 0; i < bufs.length; i++) {
      ByteBuffer b = bufs[i];
      if (b != null && !b.isDirect()) {
        if (out == bufs) {
          out = bufs.clone();
        }
        ByteBuffer copy = ByteBuffer.allocateDirect(b.remaining());
        copy.put(b.duplicate());
        copy.flip();
        out[i] = copy;
      }
    }
    return out;
  }

  /**
   * FileStore.getChecksumsForRanges (FileStore.java:567-595) over a file image in a direct buffer -- a
   * MappedByteBuffer of the file, whose capacity is the file length (ambrycrc_range_checksums_host):
   * checksum i = CRC-32 of bytes [first[i], second[i]), truncated at the end of the image and empty past it,
   * as the reference's FileChannel read gives them. Returned as unsigned values, the numbers the reference
   * renders with Long.toString. A range with first < 0, second < 0 or first > second throws
   * IllegalArgumentException and computes nothing. device < 0: the library's CPU threads; otherwise its
   * host-resident dispatch on that (initialised) GPU.
   */
  public static long[] rangeChecksums(ByteBuffer file, long[] first, long[] second, int device) {
    int[] out = new int[first.length];
    nativeRangeChecksums(file, first, second, out, device);
    long[] values = new long[out.length];
    for (int i = 0; i < out.length; i++) {
      values[i] = out[i] & 0xffffffffL;
    }
    return values;
  }

  /** Host-resident dispatch policies (ambrycrc_set_host_policy): auto, always the GPU, always the CPU leg. */
  public static final int HOST_AUTO = 0;
  public static final int HOST_GPU = 1;
  public static final int HOST_CPU = 2;

  /**
   * Sets how batch / verifyMessages / transformMessages on `device` run host-resident bytes (HOST_AUTO: the
   * CPU leg for pageable bytes when its threads beat the GPU host path, see hostRates); returns the
   * previous policy. Throws IllegalStateException for a device not initialised, IllegalArgumentException
   * for an unknown policy.
   */
  public static int setHostPolicy(int device, int policy) {
    return nativeSetHostPolicy(device, policy);
  }

  /**
   * The rates HOST_AUTO compares on `device`: {CPU leg GiB/s, GPU host path GiB/s, CPU threads}
   * (ambrycrc_host_rates).
   */
  public static double[] hostRates(int device) {
    double[] out = new double[3];
    nativeHostRates(device, out);
    return out;
  }

  /**
   * The CPU leg's thread budget on `device` (-1: the process's; 0: the default, half the CPUs this process may
   * use, leaving the rest to the server's network and disk threads) -- ambrycrc_set_host_cpu_threads. HOST_AUTO
   * rates the CPU leg at this budget. Returns the previous setting.
   */
  public static int setHostCpuThreads(int device, int threads) {
    return nativeSetHostCpuThreads(device, threads);
  }

  /** The leg `device`'s last host-resident call took: 0 the CPU, 1 the GPU, -1 none yet. */
  public static int lastHostPath(int device) {
    return nativeLastHostPath(device);
  }

  /** AMBRYCRC_MSG_* status bits of verifyMessages (include/ambrycrc.h). */
  public static final int MSG_HEADER_CRC = 1;
  public static final int MSG_ENCKEY_CRC = 1 << 1;
  public static final int MSG_PROPS_CRC = 1 << 2;
  public static final int MSG_UPDATE_CRC = 1 << 3;
  public static final int MSG_USERMETA_CRC = 1 << 4;
  public static final int MSG_BLOB_CRC = 1 << 5;
  public static final int MSG_BAD_VERSION = 1 << 8;
  public static final int MSG_BAD_LAYOUT = 1 << 9;
  public static final int MSG_NOT_PUT = 1 << 10;
  public static final int MSG_BAD_RECORD = 1 << 11;
  public static final int MSG_NO_ROOM = 1 << 12;
  /** A BlobProperties string is not ASCII: the reference's V5 re-serialization overflows its buffer. */
  public static final int MSG_NOT_ENCODABLE = 1 << 13;

  private static native void nativeInit(int device);

  private static native int nativeUpdateArray(int crc, byte[] b, int off, int len);

  private static native int nativeUpdateDirect(int crc, ByteBuffer buf, int pos, int len);

  private static native int nativeUpdateByte(int crc, int b);

  private static native int nativeUpdateDirectAll(int crc, ByteBuffer[] bufs);

  private static native int nativeCombine(int crc1, int crc2, long len2);

  private static native void nativeBatchDirect(ByteBuffer[] bufs, int[] pos, int[] len, int[] crcIn, int[] out,
      int device);

  private static native void nativeVerifyMessages(ByteBuffer region, long[] offsets, int[] status, long[] ends,
      int device);

  private static native int nativeVerifyMessage(ByteBuffer region, long offset, long[] end);

  private static native int nativeChainMessages(ByteBuffer region, long start, long[] offsets);

  private static native int nativeTransformMessage(ByteBuffer region, long offset, int lifeVersion,
      int headerVersion, ByteBuffer out, long[] outLen);

  private static native void nativeTransformMessages(ByteBuffer region, long[] offsets, short[] lifeVersions,
      int headerVersion, ByteBuffer out, long[] outOffsets, long[] outLens, int[] status, int device);

  private static native void nativePutCrcs(ByteBuffer[] fields, ByteBuffer[] prefixes, int[] blobCrc, long[] blobLen,
      int[] wireOut, int[] recordOut);

  private static native void nativeRangeChecksums(ByteBuffer file, long[] first, long[] second, int[] out, int device);

  private static native int nativeSetHostPolicy(int device, int policy);

  private static native int nativeHostRates(int device, double[] out);

  private static native int nativeSetHostCpuThreads(int device, int threads);

  private static native int nativeLastHostPath(int device);
}
