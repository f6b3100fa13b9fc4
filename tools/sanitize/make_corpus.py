"""Malformed-scene corpus for the sanitizer build (`make -C monte_carlo_path_tracing_amd/csrc sanitize`).

Writes (obj, xml) pairs into OUT_DIR and prints them as one argument list for tools/sanitize/san_host:
hand-written malformed OBJ / MTL / XML cases (truncated and non-numeric fields, out-of-range and zero
face indices, polygons, missing or unreadable MTL files, NaN / huge numbers, NUL bytes, CRLF, very long
lines, broken XML) plus seeded byte-level mutations of the Veach stand-in (scenes/veach-mis).  The
loaders under test are the library's (scene_io.cpp, the reference's Myobj::read / Mylight::read,
Myobj.cpp:10-28, Mylight.cpp:11-100) and the oracle's.

    python tools/sanitize/make_corpus.py OUT_DIR [n_mutants]
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SCENE = os.path.join(ROOT, "scenes", "veach-mis")

MTL = "newmtl lamp\nKd 0 0 0\nKs 0 0 0\nNs 1\nnewmtl wall\nKd 0.5 0.5 0.5\nKs 0.1 0.1 0.1\nNs 20\n"
XML = '<light mtlname="lamp" radiance="10,10,10"/>\n'
TRI = "v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\n"
GOOD_OBJ = "mtllib m.mtl\n" + TRI + "v 0 0 1\nv 1 0 1\nv 0 1 1\nusemtl wall\nf 1//1 2//1 3//1\nusemtl lamp\nf 4//1 6//1 5//1\n"

OBJ_CASES = {
    "empty": "",
    "comments": "# nothing\n#\n\n",
    "v_short": "mtllib m.mtl\nv 1 2\nv\nusemtl wall\nf 1 1 1\n",
    "v_text": "mtllib m.mtl\nv a b c\nv 1e999 -1e999 nan\nv 0x10 1e-400 --1\nusemtl wall\nf 1 2 3\n",
    "f_oob": "mtllib m.mtl\n" + TRI + "usemtl wall\nf 1 2 99\nf -9 1 2\nf 0 1 2\n",
    "f_neg": "mtllib m.mtl\n" + TRI + "usemtl wall\nf -1 -2 -3\nf -3//-1 -2//-1 -1//-1\n",
    "f_two": "mtllib m.mtl\n" + TRI + "usemtl wall\nf 1 2\nf 1\nf\n",
    "f_poly": "mtllib m.mtl\n" + TRI + "v 1 1 0\nv 2 2 0\nusemtl wall\nf 1 2 4 5 3 1 2 4 5 3 1 2\n",
    "f_slash": "mtllib m.mtl\n" + TRI + "usemtl wall\nf 1/ 2// 3///\nf 1/x/y 2/2/2 3/3/3\nf //1 //2 //3\n",
    "vn_oob": "mtllib m.mtl\n" + TRI + "usemtl wall\nf 1//7 2//-7 3//0\n",
    "no_mtllib": TRI + "usemtl wall\nf 1 2 3\n",
    "mtl_missing": "mtllib nope.mtl\n" + TRI + "usemtl wall\nf 1 2 3\n",
    "mtl_dir": "mtllib .\n" + TRI + "usemtl wall\nf 1 2 3\n",
    "usemtl_undef": "mtllib m.mtl\n" + TRI + "usemtl ghost\nf 1 2 3\n",
    "no_usemtl": "mtllib m.mtl\n" + TRI + "f 1 2 3\n",
    "nul": "mtllib m.mtl\n" + TRI + "usemtl wall\x00\nf 1\x002 3\n",
    "crlf": GOOD_OBJ.replace("\n", "\r\n"),
    "cr_only": GOOD_OBJ.replace("\n", "\r"),
    "no_final_newline": GOOD_OBJ.rstrip("\n"),
    "tabs": GOOD_OBJ.replace(" ", "\t"),
    "long_line": "mtllib m.mtl\n" + TRI + "v " + "1" * 200000 + " 2 3\nusemtl wall\nf 1 2 3\n# " + "x" * 300000 + "\n",
    "many_tokens": "mtllib m.mtl\n" + TRI + "usemtl wall\nf " + " ".join(["1", "2", "3"] * 5000) + "\n",
    "good": GOOD_OBJ,
    "degenerate": "mtllib m.mtl\nv 0 0 0\nv 0 0 0\nv 0 0 0\nvn 0 0 0\nusemtl lamp\nf 1//1 2//1 3//1\nusemtl wall\nf 1 2 3\n",
    "binary": "".join(chr(c) for c in range(256)) * 4,
}
MTL_CASES = {
    "mtl_garbage": "newmtl wall\nKd x y z\nKs 1\nNs\nnewmtl\nnewmtl lamp\nKd 1e999 nan -1\n",
    "mtl_empty": "",
    "mtl_dup": MTL + MTL,
}
XML_CASES = {
    "x_empty": "",
    "x_unclosed": '<light mtlname="lamp" radiance="10,10,10"',
    "x_noattr": "<light/>\n<light mtlname=\"lamp\"/>\n<light radiance=\"1,2,3\"/>\n",
    "x_badrad": '<light mtlname="lamp" radiance="1,2"/>\n<light mtlname="wall" radiance="a,b,c"/>\n',
    "x_huge": '<light mtlname="lamp" radiance="1e999,-1e999,nan"/>\n',
    "x_unknown": '<light mtlname="ghost" radiance="1,1,1"/>\n',
    "x_quotes": "<light mtlname=lamp radiance=10,10,10/>\n<light mtlname='lamp' radiance='1,1,1'/>\n",
    "x_nested": '<scene><light mtlname="lamp" radiance="1,1,1"><light mtlname="wall" radiance="1,1,1"/></light></scene>\n',
    "x_camera": '<camera type="perspective" width="x" height="-5" fovy="nan"><eye x="1"/><lookat/><up y="1" z="q"/></camera>\n' + XML,
    "x_long": '<light mtlname="' + "l" * 100000 + '" radiance="1,1,1"/>\n',
    "x_binary": "".join(chr(c) for c in range(256)),
    "x_good": XML,
}


def write(path, text):
    with open(path, "w", encoding="latin-1", newline="") as f:
        f.write(text)


def main():
    out = sys.argv[1]
    nmut = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    os.makedirs(out, exist_ok=True)
    write(os.path.join(out, "m.mtl"), MTL)
    pairs = []
    for name, text in OBJ_CASES.items():
        p = os.path.join(out, name + ".obj")
        write(p, text)
        pairs.append((p, os.path.join(out, "x_good.xml")))
    for name, text in XML_CASES.items():
        write(os.path.join(out, name + ".xml"), text)
        pairs.append((os.path.join(out, "good.obj"), os.path.join(out, name + ".xml")))
    for name, text in MTL_CASES.items():  # an OBJ per MTL variant, in its own directory
        d = os.path.join(out, name)
        os.makedirs(d, exist_ok=True)
        write(os.path.join(d, "m.mtl"), text)
        write(os.path.join(d, "s.obj"), GOOD_OBJ)
        pairs.append((os.path.join(d, "s.obj"), os.path.join(out, "x_good.xml")))
    # seeded byte mutations of the Veach stand-in (OBJ, MTL and XML), one file of the three per mutant
    src = {ext: open(os.path.join(SCENE, "veach-mis." + ext), "rb").read() for ext in ("obj", "mtl", "xml")}
    rng = random.Random(20240430)
    for k in range(nmut):
        d = os.path.join(out, "mut%03d" % k)
        os.makedirs(d, exist_ok=True)
        which = ("obj", "mtl", "xml")[k % 3]
        for ext, data in src.items():
            b = bytearray(data)
            if ext == which:
                for _ in range(rng.randint(1, 40)):
                    op = rng.random()
                    i = rng.randrange(len(b))
                    if op < 0.5:
                        b[i] = rng.choice(b"0123456789-+.eE/ \n\x00xv#f")
                    elif op < 0.75:
                        del b[i:i + rng.randint(1, 64)]
                    else:
                        b[i:i] = bytes(rng.choice(b"0123456789-/ \n") for _ in range(rng.randint(1, 16)))
            open(os.path.join(d, "veach-mis." + ext), "wb").write(bytes(b))
        pairs.append((os.path.join(d, "veach-mis.obj"), os.path.join(d, "veach-mis.xml")))
    pairs.append((os.path.join(SCENE, "veach-mis.obj"), os.path.join(SCENE, "veach-mis.xml")))
    print(" ".join("%s %s" % p for p in pairs))


if __name__ == "__main__":
    main()
