#!/usr/bin/env python3
"""Write a synthetic Ambry log segment for tools/verify_log.py timing: the LogSegment header and
N copies of one PUT message (V3 header, 1000 B user metadata, a random blob). The message
layout comes from oracle/message_format.py in its fixture-builder role; nothing measured runs it.
  usage: make_synthetic_log.py PATH [N messages] [blob bytes]"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    blob_bytes = int(sys.argv[3]) if len(sys.argv) > 3 else 64 << 10
    spec = importlib.util.spec_from_file_location("mf", os.path.join(ROOT, "oracle", "message_format.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    from ambry_amd import store_files

    blob = os.urandom(blob_bytes)
    tmpl = mf.put_message(mf.store_key("blob-0001"), mf.blob_properties_bytes(len(blob)), b"u" * 1000, blob)
    with open(path, "wb") as f:
        f.write(store_files.log_segment_header(1 << 40))
        for _ in range(n // 256):
            f.write(tmpl * 256)
        f.write(tmpl * (n % 256))
    print(json.dumps({"file": path, "messages": n, "bytes": os.path.getsize(path)}))


if __name__ == "__main__":
    main()
