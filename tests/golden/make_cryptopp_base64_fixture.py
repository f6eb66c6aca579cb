"""Extract tests/golden/cryptopp521_base64.json (run in the build container,
where /root/reference exists).

bitflood renders a digest with Crypto++ 5.2.1's BaseN_Encoder over the
standard base64 alphabet, 6 bits per char, no padding
(cpp/src/Encoder.cpp:104-120).  Crypto++'s own validation suite holds the
expected Base64Encoder output -- the same BaseN_Encoder with that alphabet,
plus '=' padding and a line break every 72 chars (base64.cpp:12-24) -- for the
bytes 0..254, hex-encoded (validat1.cpp:1210-1271, `base64AndHexEncoded`).
This keeps that expected output as data.
"""
import json
import os
import re

SRC = "/root/reference/cpp/extern/crypto++/5.2.1/validat1.cpp"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cryptopp521_base64.json")


def main():
    text = open(SRC, encoding="latin-1").read()
    m = re.search(r"const char \*base64AndHexEncoded = \s*((?:\"[0-9A-F]*\"\s*)+);", text)
    hexstr = "".join(re.findall(r"\"([0-9A-F]*)\"", m.group(1)))
    line = text[: m.start()].count("\n") + 1
    json.dump({"source": f"cpp/extern/crypto++/5.2.1/validat1.cpp:{line} (base64AndHexEncoded, ValidateBaseCode)",
               "input": "bytes 0..254",
               "base64_with_linebreaks": bytes.fromhex(hexstr).decode("ascii")}, open(OUT, "w"), indent=1)
    print(f"{len(hexstr) // 2} base64 chars -> {OUT}")


if __name__ == "__main__":
    main()
