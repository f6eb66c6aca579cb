"""Extract tests/golden/cryptopp521_hmac_sha1.json (run in the build container,
where /root/reference exists).

The reference's Crypto++ 5.2.1 holds HMAC(SHA-1) known answers (RFC 2202,
TestVectors/hmac.txt, the "Name: HMAC(SHA-1)" section).  HMAC is two SHA-1
passes, SHA1((K ^ opad) || SHA1((K ^ ipad) || m)) with K hashed first when it
is longer than a block, so each vector is also a known answer for SHA-1 over
messages that start with a full 64-byte block -- more reference-held answers
for the chunk-hash kernels (tests/test_oracle.py, tests/test_gpu_parity.py).
Values are kept as hex; the file's forms are 0x<hex>, "text" and r<N> <value>
(repeat N times).
"""
import json
import os
import re

SRC = "/root/reference/cpp/extern/crypto++/5.2.1/TestVectors/hmac.txt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cryptopp521_hmac_sha1.json")


def value(v: str) -> bytes:
    v = v.strip()
    m = re.match(r"r(\d+)\s+(.*)$", v)
    if m:
        return value(m.group(2)) * int(m.group(1))
    if v.startswith('"') and v.endswith('"'):
        return v[1:-1].encode()
    if v.startswith("0x"):
        return bytes.fromhex(v[2:])
    raise ValueError(v)


def main():
    lines = open(SRC, encoding="latin-1").read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.strip() == "Name: HMAC(SHA-1)")
    cases, cur = [], {}
    for i in range(start + 1, len(lines)):
        l = lines[i]
        if l.startswith("AlgorithmType:"):
            break
        k, _, v = l.partition(":")
        k = k.strip()
        if k == "Comment":
            cur = {"name": v.strip(), "line": i + 1}
        elif k in ("Key", "Message"):
            cur[k.lower()] = value(v).hex()
        elif k == "Digest" and "digest" not in cur:
            cur["digest"] = value(v).hex()
        elif k == "Test" and v.strip() == "Verify" and "digest" in cur and cur not in cases:
            cases.append(cur)
    json.dump({"source": "cpp/extern/crypto++/5.2.1/TestVectors/hmac.txt (HMAC(SHA-1), RFC 2202)", "cases": cases},
              open(OUT, "w"), indent=1)
    print(f"{len(cases)} HMAC(SHA-1) cases -> {OUT}")


if __name__ == "__main__":
    main()
