/*
 * NativeBlobStoreRecovery -- BlobStoreRecovery.recover (ambry-messageformat/.../BlobStoreRecovery.java:43-110)
 * with the record CRCs of the whole span verified by libambrycrc in batches instead of message by message
 * through CrcInputStream. integration/ambry-messageformat-batch-recovery.patch makes BlobStoreRecovery.recover
 * call it when ambry.native.recovery.device >= 0 and the span fits one direct buffer.
 *
 * The result is the reference's: the messages before the first one that fails (in log order), and for that
 * message a StoreException(LogFileFormatError) with startOffset left at its first byte; a span that parses to
 * its end returns no exception and startOffset = endOffset. What runs where:
 *   - the hop from header to header (version, header CRC, sizes): NativeCrc32.chainMessages, on the CPU;
 *   - every record CRC of the chained messages (header, encryption key, properties, update, user metadata,
 *     blob): NativeCrc32.verifyMessages, one call per 65,536 messages, on the GPU `device`;
 *   - the MessageInfo of each clean message: the reference's own code on the small records it reads them
 *     from (key, blob properties or update record, ~100 B; their CRCs are checked again there), so the
 *     fields, sizes and exceptions are the reference's.
 */
package com.github.ambry.messageformat;

import com.github.ambry.store.MessageInfo;
import com.github.ambry.store.MessageStoreRecovery;
import com.github.ambry.store.Read;
import com.github.ambry.store.StoreErrorCodes;
import com.github.ambry.store.StoreException;
import com.github.ambry.store.StoreKey;
import com.github.ambry.store.StoreKeyFactory;
import com.github.ambry.utils.ByteBufferInputStream;
import com.github.ambry.utils.NativeCrc32;
import com.github.ambry.utils.Utils;
import java.io.DataInputStream;
import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.Arrays;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;

import static com.github.ambry.messageformat.MessageFormatRecord.*;


public class NativeBlobStoreRecovery {
  private static final Logger logger = LoggerFactory.getLogger(NativeBlobStoreRecovery.class);
  /** GPU of the batch verify; -1 (the default) leaves recovery to the reference loop. */
  static final int DEVICE = Integer.getInteger("ambry.native.recovery.device", -1);
  /** Spans up to this many bytes are read whole into one direct buffer; longer ones take the reference loop. */
  static final long MAX_SPAN = Math.min(Long.getLong("ambry.native.recovery.max.span", 1L << 30), Integer.MAX_VALUE);
  /** Messages per chain / verify call. */
  static final int BATCH = 1 << 16;

  static boolean applies(long startOffset, long endOffset) {
    return DEVICE >= 0 && startOffset < endOffset && endOffset - startOffset <= MAX_SPAN;
  }

  static MessageStoreRecovery.RecoveryResult recover(Read read, long startOffset, long endOffset,
      StoreKeyFactory factory) {
    NativeCrc32.init(DEVICE);
    ArrayList<MessageInfo> messageRecovered = new ArrayList<>();
    StoreException recoveryException = null;
    long span = endOffset - startOffset;
    long pos = 0;  // span-relative start of the next message; startOffset + pos is the reference's startOffset
    try {
      ByteBuffer region = ByteBuffer.allocateDirect((int) span);
      read.readInto(region, startOffset);
      long[] offsets = new long[BATCH];
      while (pos < span) {
        int n = NativeCrc32.chainMessages(region, pos, offsets);
        if (n == 0) {
          // the header at pos does not parse (version, verifyHeader, sizes) or its message runs past endOffset:
          // where the reference's loop throws
          throw new MessageFormatException("Message at " + (startOffset + pos) + " cannot be recovered",
              MessageFormatErrorCodes.DataCorrupt);
        }
        long[] offs = Arrays.copyOf(offsets, n);
        int[] status = new int[n];
        long[] ends = new long[n];
        NativeCrc32.verifyMessages(region, offs, status, ends, DEVICE);
        for (int k = 0; k < n; k++) {
          if (status[k] != 0) {
            throw new MessageFormatException(
                "Message at " + (startOffset + offs[k]) + " failed verification, status 0x" + Integer.toHexString(
                    status[k]), MessageFormatErrorCodes.DataCorrupt);
          }
          messageRecovered.add(messageInfo(region, offs[k], ends[k], factory));
          pos = ends[k];
        }
      }
    } catch (MessageFormatException | IndexOutOfBoundsException e) {
      logger.error("Message format exception while recovering messages, startOffset is {}, endOffset is {}",
          startOffset + pos, endOffset, e);
      recoveryException = new StoreException(e, StoreErrorCodes.LogFileFormatError);
    } catch (Throwable throwable) {
      logger.error("Unexpected exception, startOffset is {}, endOffset is {}", startOffset + pos, endOffset);
      recoveryException = throwable instanceof StoreException ? (StoreException) throwable
          : new StoreException(throwable, StoreErrorCodes.LogFileFormatError);
    }
    return new MessageStoreRecovery.RecoveryResult(messageRecovered, recoveryException, startOffset + pos);
  }

  /**
   * The MessageInfo BlobStoreRecovery.recover builds for the verified message at region[off, end): the key, and
   * the blob properties (a put) or the update record (anything else), read by the reference's deserializers.
   */
  private static MessageInfo messageInfo(ByteBuffer region, long off, long end, StoreKeyFactory factory)
      throws IOException, MessageFormatException {
    if (off < 0 || end > region.capacity() || off >= end) {
      throw new IndexOutOfBoundsException("message [" + off + ", " + end + ") outside the span");
    }
    ByteBuffer msg = slice(region, off, end);
    short version = msg.getShort(0);
    ByteBuffer header = slice(msg, 0, getHeaderSizeForVersion(version));
    MessageHeader_Format headerFormat = getMessageHeader(version, header);
    StoreKey key = factory.getStoreKey(
        new DataInputStream(new ByteBufferInputStream(slice(msg, header.capacity(), msg.capacity()))));
    short lifeVersion = headerFormat.hasLifeVersion() ? headerFormat.getLifeVersion() : 0;
    long size = header.capacity() + key.sizeInBytes() + headerFormat.getMessageSize();
    if (headerFormat.isPutRecord()) {
      BlobProperties properties = deserializeBlobProperties(
          new ByteBufferInputStream(slice(msg, headerFormat.getBlobPropertiesRecordRelativeOffset(), msg.capacity())));
      return new MessageInfo(key, size, false, false, false,
          Utils.addSecondsToEpochTime(properties.getCreationTimeInMs(), properties.getTimeToLiveInSeconds()), null,
          properties.getAccountId(), properties.getContainerId(), properties.getCreationTimeInMs(), lifeVersion);
    }
    UpdateRecord updateRecord = deserializeUpdateRecord(
        new ByteBufferInputStream(slice(msg, headerFormat.getUpdateRecordRelativeOffset(), msg.capacity())));
    boolean deleted = false, ttlUpdated = false, undeleted = false;
    switch (updateRecord.getType()) {
      case DELETE:
        deleted = true;
        break;
      case TTL_UPDATE:
        ttlUpdated = true;
        break;
      case UNDELETE:
        undeleted = true;
        break;
      default:
        throw new IllegalStateException("Unknown update record type: " + updateRecord.getType());
    }
    return new MessageInfo(key, size, deleted, ttlUpdated, undeleted, updateRecord.getAccountId(),
        updateRecord.getContainerId(), updateRecord.getUpdateTimeInMs(), lifeVersion);
  }

  private static ByteBuffer slice(ByteBuffer b, long from, long to) {
    ByteBuffer d = b.duplicate();
    d.limit((int) to).position((int) from);
    return d.slice();
  }
}
