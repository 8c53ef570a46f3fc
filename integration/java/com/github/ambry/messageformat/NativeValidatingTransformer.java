/*
 * NativeValidatingTransformer -- drop-in for ValidatingTransformer
 * (ambry-messageformat/.../messageformat/ValidatingTransformer.java:37-104) backed by libambrycrc:
 * the deserialize-verify-reserialize of a stored PUT runs in C (ambrycrc_transform_message_cpu, one
 * message) or on the GPU (ambrycrc_transform_messages_host, a whole GetResponse), with every CRC
 * recomputed the way PutMessageFormatInputStream writes it. Selected like the reference transformer,
 * by class name: server.message.transformer (ServerConfig.java:66-68) =
 * com.github.ambry.messageformat.NativeValidatingTransformer (INTEGRATION.md).
 *
 * What stays in Java: the StoreKey comparison with the index entry (ValidatingTransformer.java:
 * 80-98), MessageInfo bookkeeping, and mapping the library's status bits to the exceptions the
 * reference wraps in TransformationOutput(e) -- MessageFormatException for corrupt data (the
 * message is then skipped by MessageSievingInputStream.java:296-302), IllegalStateException for an
 * update record or a key mismatch, BufferOverflowException for a property string PutMessageFormat-
 * InputStream cannot re-encode (both abort the batch there, :303-305).
 */
package com.github.ambry.messageformat;

import com.github.ambry.store.Message;
import com.github.ambry.store.MessageInfo;
import com.github.ambry.store.StoreKey;
import com.github.ambry.store.StoreKeyConverter;
import com.github.ambry.store.StoreKeyFactory;
import com.github.ambry.store.TransformationOutput;
import com.github.ambry.store.Transformer;
import com.github.ambry.utils.ByteBufferInputStream;
import com.github.ambry.utils.NativeCrc32;
import com.github.ambry.utils.Utils;
import java.io.DataInputStream;
import java.io.IOException;
import java.nio.BufferOverflowException;
import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;


public class NativeValidatingTransformer implements Transformer {
  private final StoreKeyFactory storeKeyFactory;
  /** GPU of transformAll (-1: the per-message CPU path for batches too). */
  private final int device;

  /** Same constructor as ValidatingTransformer, so Utils.getObj can build it from the config. */
  public NativeValidatingTransformer(StoreKeyFactory storeKeyFactory, StoreKeyConverter storeKeyConverter) {
    this(storeKeyFactory, storeKeyConverter, Integer.getInteger("ambry.native.transform.device", 0));
  }

  public NativeValidatingTransformer(StoreKeyFactory storeKeyFactory, StoreKeyConverter storeKeyConverter,
      int device) {
    this.storeKeyFactory = storeKeyFactory;
    this.device = device;
    if (device >= 0) {
      NativeCrc32.init(device);
    }
  }

  /** ValidatingTransformer.transform (ValidatingTransformer.java:46-104), one message, on the CPU. */
  @Override
  public TransformationOutput transform(Message message) {
    MessageInfo msgInfo = message.getMessageInfo();
    try {
      if (NativeCrc32.transformOutBound(msgInfo.getSize(), 1) > Integer.MAX_VALUE) {
        throw new IOException("message of " + msgInfo.getSize() + " bytes: past a direct buffer's reach");
      }
      int size = (int) msgInfo.getSize();
      ByteBuffer in = ByteBuffer.allocateDirect(size);
      in.put(Utils.readBytesFromStream(message.getStream(), size));
      ByteBuffer out = ByteBuffer.allocateDirect((int) NativeCrc32.transformOutBound(size, 1));
      long[] outLen = new long[1];
      int status = NativeCrc32.transformMessage(in, 0, msgInfo.getLifeVersion(),
          MessageFormatRecord.getCurrentMessageHeaderVersion(), out, outLen);
      return output(msgInfo, status, in, 0, out, 0, outLen[0]);
    } catch (Exception e) {
      return new TransformationOutput(e);
    }
  }

  /**
   * transform() over every message of one GetResponse at once, on the GPU: `region` (direct) holds
   * the messages back to back as MessageSievingInputStream reads them (MessageSievingInputStream.java:
   * 112-130); messages the sieve skips (deleted, expired) get a null entry. One native call for the
   * batch; the outputs are slices of one direct buffer.
   */
  public List<TransformationOutput> transformAll(ByteBuffer region, List<MessageInfo> infos) throws IOException {
    List<TransformationOutput> result = new ArrayList<>(infos.size());
    List<Integer> live = new ArrayList<>();
    long[] starts = new long[infos.size()];
    long at = 0;
    for (int i = 0; i < infos.size(); i++) {
      MessageInfo info = infos.get(i);
      starts[i] = at;
      at += info.getSize();
      result.add(null);
      if (!info.isDeleted() && !info.isExpired()) {
        live.add(i);
      }
    }
    if (at > region.capacity()) {
      throw new IOException("GetResponse region holds " + region.capacity() + " bytes, message infos " + at);
    }
    // every offset below is < at <= capacity (an int); the output bound is checked before its allocation
    if (device < 0) {
      for (int i : live) {
        ByteBuffer msg = region.duplicate();
        msg.position((int) starts[i]).limit((int) (starts[i] + infos.get(i).getSize()));
        result.set(i, transform(new Message(infos.get(i), new ByteBufferInputStream(msg.slice()))));
      }
      return result;
    }
    int m = live.size();
    long[] offsets = new long[m];
    short[] life = new short[m];
    long bytes = 0;
    for (int k = 0; k < m; k++) {
      MessageInfo info = infos.get(live.get(k));
      offsets[k] = starts[live.get(k)];
      life[k] = info.getLifeVersion();
      bytes += info.getSize();
    }
    long bound = NativeCrc32.transformOutBound(bytes, m);
    if (bound > Integer.MAX_VALUE) {
      throw new IOException("transform output bound " + bound + " B: past a direct buffer's reach; split the batch");
    }
    ByteBuffer out = ByteBuffer.allocateDirect((int) bound);
    long[] outOffsets = new long[m];
    long[] outLens = new long[m];
    int[] status = new int[m];
    NativeCrc32.transformMessages(region, offsets, life, MessageFormatRecord.getCurrentMessageHeaderVersion(), out,
        outOffsets, outLens, status, device);
    for (int k = 0; k < m; k++) {
      int i = live.get(k);
      try {
        result.set(i, output(infos.get(i), status[k], region, offsets[k], out, outOffsets[k], outLens[k]));
      } catch (Exception e) {
        result.set(i, new TransformationOutput(e));
      }
    }
    return result;
  }

  @Override
  public void warmup(List<MessageInfo> messageInfos, boolean includeAll) {
    // no-op, as ValidatingTransformer.warmup
  }

  /**
   * The reference's outcome for a message whose native status is `status`: the stored message is at
   * `in`[inOff..], its re-serialization at `out`[outOff, outOff + outLen).
   */
  private TransformationOutput output(MessageInfo msgInfo, int status, ByteBuffer in, long inOff, ByteBuffer out,
      long outOff, long outLen) throws Exception {
    if (status != 0) {
      throw exceptionFor(status, in, (int) inOff);
    }
    ByteBuffer msg = out.duplicate();
    msg.position((int) outOff).limit((int) (outOff + outLen));
    msg = msg.slice();
    // the StoreKey comparison stays here: keyInStream sits right after the output header
    ByteBuffer key = msg.duplicate();
    key.position(MessageFormatRecord.getHeaderSizeForVersion(key.getShort(0)));
    StoreKey keyInStream = storeKeyFactory.getStoreKey(new DataInputStream(new ByteBufferInputStream(key.slice())));
    if (!msgInfo.getStoreKey().equals(keyInStream)) {
      throw new IllegalStateException(
          "StoreKey in stream: " + keyInStream + " failed to match store key from Index: " + msgInfo.getStoreKey());
    }
    MessageInfo transformedMsgInfo =
        new MessageInfo.Builder(msgInfo).size(outLen).isDeleted(false).isUndeleted(false).build();
    return new TransformationOutput(new Message(transformedMsgInfo, new ByteBufferInputStream(msg)));
  }

  /**
   * The exception ValidatingTransformer would have caught, in its order of checks: the header
   * version, verifyHeader and the header constraints (MessageFormatException), the put/update shape
   * (IllegalStateException), then the record deserializers in record order (the lowest record bit:
   * UnknownFormatVersion for a bad record version, DataCorrupt otherwise), then the V5 re-encoding.
   */
  static Exception exceptionFor(int status, ByteBuffer in, int off) {
    short version = in.capacity() - off >= 2 ? in.getShort(off) : -1;
    if (version < 1 || version > 3) {
      return new MessageFormatException("Header version not supported " + version,
          MessageFormatErrorCodes.DataCorrupt);
    }
    if ((status & NativeCrc32.MSG_HEADER_CRC) != 0) {
      return new MessageFormatException("Message header is corrupt", MessageFormatErrorCodes.DataCorrupt);
    }
    if ((status & NativeCrc32.MSG_BAD_LAYOUT) != 0) {
      return new MessageFormatException("Message header constraints are violated",
          MessageFormatErrorCodes.HeaderConstraintError);
    }
    // the update record's relative offset: -1 in a put (V1 at 14, V2 at 18, V3 at 20)
    int updateAt = off + (version == 1 ? 14 : version == 2 ? 18 : 20);
    if ((status & NativeCrc32.MSG_NOT_PUT) != 0 || in.getInt(updateAt) != -1) {
      return new IllegalStateException("Message cannot be anything rather than put record ");
    }
    int[] records = {NativeCrc32.MSG_ENCKEY_CRC, NativeCrc32.MSG_PROPS_CRC, NativeCrc32.MSG_USERMETA_CRC,
        NativeCrc32.MSG_BLOB_CRC};
    for (int bit : records) {
      if ((status & bit) != 0) {
        return new MessageFormatException("corrupt data while parsing a record (CRC)",
            MessageFormatErrorCodes.DataCorrupt);
      }
    }
    if ((status & NativeCrc32.MSG_BAD_VERSION) != 0) {
      return new MessageFormatException("record version not supported", MessageFormatErrorCodes.UnknownFormatVersion);
    }
    if ((status & NativeCrc32.MSG_BAD_RECORD) != 0) {
      return new MessageFormatException("corrupt data while parsing a record", MessageFormatErrorCodes.DataCorrupt);
    }
    if ((status & NativeCrc32.MSG_NOT_ENCODABLE) != 0) {
      return new BufferOverflowException();
    }
    return new IllegalStateException("native transform status 0x" + Integer.toHexString(status));
  }
}
