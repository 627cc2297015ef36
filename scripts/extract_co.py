"""Extract the gfx950 code object (the one holding SYMBOL, default any) from an in-tree HIP shared library (clang
offload bundle in .hip_fatbin) so llvm-readelf / llvm-objdump can report
per-kernel register counts, spills and LDS.  Usage: extract_co.py LIB OUT [SYMBOL]"""
import struct
import sys

data = open(sys.argv[1], "rb").read()
magic = b"__CLANG_OFFLOAD_BUNDLE__"
pos = data.find(magic)
while pos >= 0:
    n = struct.unpack_from("<Q", data, pos + 24)[0]
    p = pos + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", data, p)
        triple = data[p + 24:p + 24 + tl].decode()
        p += 24 + tl
        blob = data[pos + off:pos + off + size]
        if "gfx950" in triple and (len(sys.argv) < 4 or sys.argv[3].encode() in blob):
            open(sys.argv[2], "wb").write(blob)
            print(triple, size)
            sys.exit(0)
    pos = data.find(magic, pos + 1)
sys.exit("no gfx950 code object")
