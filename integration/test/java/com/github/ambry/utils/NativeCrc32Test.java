/*
 * NativeCrc32Test -- JUnit 4 checks a maintainer runs in ambry-utils after adding NativeCrc32:
 * same values as java.util.zip.CRC32 and Crc32 for arrays, heap / direct / read-only buffers,
 * split updates, single bytes, gather lists and combine; out-of-bounds arguments throw.
 * (Invariants of Crc32Test / CrcInputStreamTest / CrcOutputStreamTest; SURVEY.md §8c.)
 */
package com.github.ambry.utils;

import java.nio.ByteBuffer;
import java.util.Random;
import java.util.zip.CRC32;
import org.junit.Test;

import static org.junit.Assert.*;


public class NativeCrc32Test {
  private static long jdk(byte[] b, int off, int len) {
    CRC32 c = new CRC32();
    c.update(b, off, len);
    return c.getValue();
  }

  @Test
  public void matchesJdkAndCrc32() {
    Random r = new Random(20261016);
    for (int len : new int[]{0, 1, 7, 63, 64, 65, 1000, 4096, 65539, 4 << 20}) {
      byte[] b = new byte[len + 3];
      r.nextBytes(b);
      NativeCrc32 n = new NativeCrc32();
      n.update(b, 3, len);
      Crc32 ref = new Crc32();
      ref.update(b, 3, len);
      assertEquals(jdk(b, 3, len), n.getValue());
      assertEquals(ref.getValue(), n.getValue());
    }
    NativeCrc32 n = new NativeCrc32();
    n.update("123456789".getBytes(), 0, 9);
    assertEquals(0xCBF43926L, n.getValue());
  }

  @Test
  public void buffersAreConsumedLikeCrc32() {
    byte[] b = new byte[100000];
    new Random(1).nextBytes(b);
    long want = jdk(b, 17, 90000);
    for (ByteBuffer buf : new ByteBuffer[]{ByteBuffer.wrap(b), ByteBuffer.allocateDirect(b.length),
        ByteBuffer.wrap(b).asReadOnlyBuffer()}) {
      if (buf.isDirect()) {
        buf.put(b).flip();
      }
      buf.position(17).limit(17 + 90000);
      NativeCrc32 n = new NativeCrc32();
      n.update(buf);
      assertEquals(want, n.getValue());
      assertEquals(buf.limit(), buf.position());
    }
  }

  @Test
  public void splitUpdatesEqualOneUpdate() {
    byte[] b = new byte[5000];
    new Random(2).nextBytes(b);
    NativeCrc32 n = new NativeCrc32();
    for (int i = 0; i < b.length; i += 333) {
      n.update(b, i, Math.min(333, b.length - i));
    }
    NativeCrc32 bytes = new NativeCrc32();
    for (byte x : b) {
      bytes.update(x);
    }
    assertEquals(jdk(b, 0, b.length), n.getValue());
    assertEquals(jdk(b, 0, b.length), bytes.getValue());
    long a = jdk(b, 0, 1234), c = jdk(b, 1234, b.length - 1234);
    assertEquals(jdk(b, 0, b.length), NativeCrc32.combine(a, c, b.length - 1234));
  }

  @Test
  public void gatherListOfDirectBuffers() {
    byte[] b = new byte[3 * 4096];
    new Random(3).nextBytes(b);
    ByteBuffer[] parts = new ByteBuffer[3];
    for (int i = 0; i < 3; i++) {
      parts[i] = ByteBuffer.allocateDirect(4096);
      parts[i].put(b, i * 4096, 4096).flip();
    }
    NativeCrc32 n = new NativeCrc32();
    n.updateAll(parts);
    assertEquals(jdk(b, 0, b.length), n.getValue());
  }

  @Test
  public void badArgumentsThrowAndLeaveTheValue() {
    NativeCrc32 n = new NativeCrc32();
    n.update(new byte[]{1, 2, 3}, 0, 3);
    long v = n.getValue();
    try {
      n.update(new byte[4], 2, 3);
      fail();
    } catch (ArrayIndexOutOfBoundsException expected) {
    }
    try {
      n.update(new byte[4], -1, 1);
      fail();
    } catch (ArrayIndexOutOfBoundsException expected) {
    }
    assertEquals(v, n.getValue());
  }

  /**
   * With ambry-utils-crc32-native.patch applied, Crc32 itself delegates updates of CRC32_MIN_BYTES and more to the
   * library: the same values as java.util.zip.CRC32 across the threshold, for arrays and heap / direct / read-only
   * buffers (consumed), in pieces straddling it, and the same exception for a bad range with the value unchanged.
   */
  @Test
  public void crc32DelegatesAcrossTheThreshold() {
    assertTrue(NativeCrc32.isAvailable());
    int t = NativeCrc32.CRC32_MIN_BYTES;
    byte[] b = new byte[4 * t + 11];
    new Random(7).nextBytes(b);
    for (int len : new int[]{t - 1, t, t + 1, 4 * t}) {
      Crc32 c = new Crc32();
      c.update(b, 5, len);
      assertEquals(jdk(b, 5, len), c.getValue());
      for (ByteBuffer buf : new ByteBuffer[]{ByteBuffer.wrap(b), ByteBuffer.allocateDirect(b.length),
          ByteBuffer.wrap(b).asReadOnlyBuffer()}) {
        if (buf.isDirect()) {
          buf.put(b).flip();
        }
        buf.position(5).limit(5 + len);
        Crc32 d = new Crc32();
        d.update(buf);
        assertEquals(jdk(b, 5, len), d.getValue());
        assertEquals(buf.limit(), buf.position());
      }
    }
    Crc32 pieces = new Crc32();
    pieces.update(b, 0, 3);
    pieces.update(b, 3, t + 2);
    pieces.update(b[t + 5]);
    pieces.update(b, t + 6, b.length - t - 6);
    assertEquals(jdk(b, 0, b.length), pieces.getValue());
    long before = pieces.getValue();
    try {
      pieces.update(b, b.length - t + 1, t);
      fail("expected ArrayIndexOutOfBoundsException");
    } catch (ArrayIndexOutOfBoundsException e) {
      assertEquals(before, pieces.getValue());
    }
  }
}
