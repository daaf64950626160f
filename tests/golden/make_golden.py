"""Generates tests/golden/kat.json: known-answer vectors transcribed (as data) from the reference's
own tests, each tagged with the file:line it comes from.  Paths are relative to
/root/reference/codec-compression/src/test/java/io/netty/handler/codec/compression/ unless absolute.

Run: python tests/golden/make_golden.py   (no reference access needed: the vectors are inline data)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def b(*xs):
    return bytes([x & 0xFF for x in xs]).hex()


NETTY = [0x6e, 0x65, 0x74, 0x74, 0x79]
STREAM = [0xff, 0x06, 0x00, 0x00, 0x73, 0x4e, 0x61, 0x50, 0x70, 0x59]
LONG_TEXT = ("Netty has been designed carefully with the experiences earned from the implementation of a lot of "
             "protocols such as FTP, SMTP, HTTP, and various binary and text-based legacy protocols")
LONG_TEXT_ENC = [
    -0x49, 0x01, -0x10, 0x42,
    0x4e, 0x65, 0x74, 0x74, 0x79, 0x20, 0x68, 0x61, 0x73, 0x20, 0x62, 0x65, 0x65, 0x6e, 0x20, 0x64, 0x65, 0x73, 0x69, 0x67,
    0x6e, 0x65, 0x64, 0x20, 0x63, 0x61, 0x72, 0x65, 0x66, 0x75, 0x6c, 0x6c, 0x79, 0x20, 0x77, 0x69, 0x74, 0x68, 0x20, 0x74,
    0x68, 0x65, 0x20, 0x65, 0x78, 0x70, 0x65, 0x72, 0x69, 0x65, 0x6e, 0x63, 0x65, 0x73, 0x20, 0x65, 0x61, 0x72, 0x6e, 0x65,
    0x64, 0x20, 0x66, 0x72, 0x6f, 0x6d, 0x20,
    0x01, 0x1c, 0x58,
    0x69, 0x6d, 0x70, 0x6c, 0x65, 0x6d, 0x65, 0x6e, 0x74, 0x61, 0x74, 0x69, 0x6f, 0x6e, 0x20, 0x6f, 0x66, 0x20, 0x61, 0x20,
    0x6c, 0x6f, 0x74,
    0x01, 0x09, 0x60,
    0x70, 0x72, 0x6f, 0x74, 0x6f, 0x63, 0x6f, 0x6c, 0x73, 0x20, 0x73, 0x75, 0x63, 0x68, 0x20, 0x61, 0x73, 0x20, 0x46, 0x54,
    0x50, 0x2c, 0x20, 0x53, 0x4d,
    0x01, 0x06, 0x04,
    0x48, 0x54,
    0x01, 0x06, 0x44,
    0x61, 0x6e, 0x64, 0x20, 0x76, 0x61, 0x72, 0x69, 0x6f, 0x75, 0x73, 0x20, 0x62, 0x69, 0x6e, 0x61, 0x72, 0x79,
    0x05, 0x13, 0x48,
    0x74, 0x65, 0x78, 0x74, 0x2d, 0x62, 0x61, 0x73, 0x65, 0x64, 0x20, 0x6c, 0x65, 0x67, 0x61, 0x63, 0x79, 0x20, 0x70,
    0x11, 0x4c,
]
ISSUE_1002 = [
    11, 0, 0, 0, 0, 0, 16, 65, 96, 119, -22, 79, -43, 76, -75, -93, 11, 104, 96, -99, 126, -98, 27, -36, 40, 117, -65, -3, -57,
    -83, -58, 7, 114, -14, 68, -122, 124, 88, 118, 54, 45, -26, 117, 13, -45, -9, 60, -73, -53, -44, 53, 68, -77, -71, 109, 43,
    -38, 59, 100, -12, -87, 44, -106, 123, -107, 38, 13, -117, -23, -49, 29, 21, 26, 66, 1] + [-1] * 65 + [
    66, 0, -104, -49, 16, -120, 22, 8, -52, -54, -102, -52, -119, -124, -92, -71, 101, -120, -52, -48, 45, -26, -24, 26, 41,
    -13, 36, 64, -47, 15, -124, -7, -16, 91, 96, 0, -93, -42, 101, 20, -74, 39, -124, 35, 43, -49, -21, -92, -20, -41, 79, 41,
    110, -105, 42, -96, 90, -9, -100, -22, -62, 91, 2, 35, 113, 117, -71, 66, 1] + [-1] * 65


def main():
    kat = {
        "snappy_decode": [
            {"src": "SnappyTest.java:41-59", "in": b(0x05, 0x10, *NETTY), "status": 0, "out": b(*NETTY)},
            {"src": "SnappyTest.java:61-82", "in": b(0x0a, 0x10, *NETTY, 0x05, 0x05), "status": 0, "out": b(*NETTY, *NETTY)},
            {"src": "SnappyTest.java:84-105", "in": b(0x0b, 0x10, *NETTY, 0x15, 0x00), "status": "OFFSET_ZERO"},
            {"src": "SnappyTest.java:107-128", "in": b(0x0a, 0x10, *NETTY, 0x15, 0x0b), "status": "OFFSET_BEYOND"},
            {"src": "SnappyTest.java:130-149", "in": b(-0x80, -0x80, -0x80, -0x80, 0x7f, 0x10, *NETTY),
             "status": "PREAMBLE_TOO_LONG"},
            {"src": "SnappyTest.java:326-359", "in": b(0x82, 0x80, 0x02, 61 << 2, 0x00, 0x80, 0x01, *([0] * 0x8000), 0x02, 0x01, 0x80),
             "status": 0, "out": b(0x01, *([0] * 0x8000), 0x01)},
        ],
        "snappy_encode": [
            {"src": "SnappyTest.java:151-169", "in": b(*NETTY), "out": b(0x05, 0x10, *NETTY)},
            {"src": "SnappyTest.java:171-248", "in": LONG_TEXT.encode("ascii").hex(), "out": b(*LONG_TEXT_ENC)},
        ],
        "snappy_literal_lengths": {"src": "SnappyTest.java:298-324", "lengths": [0x11, 0x100, 0x1000, 0x100000, 0x1000001]},
        "crc32c": [
            {"src": "SnappyTest.java:250-258", "in": b"netty".hex(), "crc": 0xd6cb8b55},
            {"src": "SnappyTest.java:283-296 (validateChecksum mismatch uses 0xd6cb8b55 for 'ytten')", "in": b"ytten".hex(),
             "crc": 0x2d4d3535},
        ],
        "masked_checksum": [
            {"src": "SnappyTest.java:260-270", "in": b(0, 0, 0, 0x0f, 0, 0, 0, 0, 0x5f, 0x68, 0x65, 0x61, 0x72, 0x74, 0x62, 0x65,
                                                     0x61, 0x74, 0x5f), "masked": 0x44a4301f},
            {"src": "/root/reference/codec-http/src/test/java/io/netty/handler/codec/http/HttpContentDecoderTest.java:57-60",
             "in": b"hello, world".hex(), "masked": 0xeac1be0b},
        ],
        "snappy_frame_encode": [
            {"src": "SnappyFrameEncoderTest.java:35-52", "msgs": [b(*NETTY)],
             "out": b(*STREAM, 0x01, 0x09, 0x00, 0x00, 0x6f, -0x68, 0x2e, -0x47, *NETTY)},
            {"src": "SnappyFrameEncoderTest.java:54-76", "msgs": [b(*(NETTY * 4))],
             "out": b(*STREAM, 0x00, 0x0E, 0x00, 0x00, 0x3b, 0x36, -0x7f, 0x37, 0x14, 0x10, *NETTY, 0x3a, 0x05, 0x00)},
            {"src": "SnappyFrameEncoderTest.java:78-107", "msgs": [b(*NETTY), b(*NETTY)],
             "out": b(*STREAM, 0x01, 0x09, 0x00, 0x00, 0x6f, -0x68, 0x2e, -0x47, *NETTY,
                      0x01, 0x09, 0x00, 0x00, 0x6f, -0x68, 0x2e, -0x47, *NETTY)},
        ],
        "snappy_frame_decode": [
            {"src": "SnappyFrameDecoderTest.java:50-61", "in": b(0x03, 0x01, 0x00, 0x00, 0x00), "error": True},
            {"src": "SnappyFrameDecoderTest.java:63-74", "in": b(-0x80, 0x05, 0x00, 0x00, *NETTY), "error": True},
            {"src": "SnappyFrameDecoderTest.java:76-87", "in": b(0xff, 0x06, 0x00, 0x00, 0x73, *NETTY), "error": True},
            {"src": "SnappyFrameDecoderTest.java:89-100", "in": b(-0x7f, 0x06, 0x00, 0x00, 0x73, *NETTY), "error": True},
            {"src": "SnappyFrameDecoderTest.java:102-114", "in": b(0x01, 0x05, 0x00, 0x00, *NETTY), "error": True},
            {"src": "SnappyFrameDecoderTest.java:116-127", "in": b(0x00, 0x05, 0x00, 0x00, *NETTY), "error": True},
            {"src": "SnappyFrameDecoderTest.java:129-139", "in": b(*STREAM, -0x7f, 0x05, 0x00, 0x00, *NETTY), "msgs": []},
            {"src": "SnappyFrameDecoderTest.java:141-155",
             "in": b(*STREAM, 0x01, 0x09, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, *NETTY), "msgs": [b(*NETTY)]},
            {"src": "SnappyFrameDecoderTest.java:157-174",
             "in": b(*STREAM, 0x00, 0x0B, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x05, 0x10, *NETTY), "msgs": [b(*NETTY)]},
            {"src": "SnappyFrameDecoderTest.java:179-199", "validate": True,
             "in": b(*STREAM, 0x01, 0x09, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, *NETTY), "error": True},
            {"src": "SnappyFrameDecoderTest.java:201-223", "validate": True,
             "in": b(*STREAM, 0x01, 0x09, 0x00, 0x00, 0x6f, -0x68, 0x2e, -0x47, *NETTY), "msgs": [b(*NETTY)]},
            {"src": "/root/reference/codec-http/src/test/java/io/netty/handler/codec/http/HttpContentDecoderTest.java:57-60",
             "validate": True,
             "in": b(-1, 6, 0, 0, 115, 78, 97, 80, 112, 89, 1, 16, 0, 0, 11, -66, -63, -22, 104, 101, 108, 108, 111, 44, 32, 119,
                     111, 114, 108, 100), "msgs": [b"hello, world".hex()]},
        ],
        "identity_inputs": {
            "src": "AbstractIntegrationTest.java:77-158, SnappyIntegrationTest.java:47-108",
            "issue_1002": b(*ISSUE_1002),
            "regular": ("Netty is a NIO client server framework which enables quick and easy development of network "
                        "applications such as protocol servers and clients.").encode().hex(),
            "snappy_seeds": [5323211032315942961, 7088170877360183401],
        },
        "java_random": {"src": "java.util.Random(42).nextInt() == -1170105035 (JDK contract)", "seed": 42,
                        "first4": "359d41ba"},
    }
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print("wrote", os.path.join(HERE, "kat.json"))


if __name__ == "__main__":
    main()
