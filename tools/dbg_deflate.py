"""Development aid (GPU box): run the record-path test inputs, save the first mismatch."""
import os, random, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from conftest import golden  # noqa: E402  (sets the oracle / package paths)
import oracle as O
import sdz
from test_gpu_parity import text_corpus, binary_corpus, _periodic, _overlay_stress
from conftest import golden

paradise = golden("paradiselost.txt")
rng = random.Random(11)
sizes = [1, 2, 3, 4, 5, 257, 258, 259, 261, 262, 263, 264, 5552, 32767, 32768, 32769,
         65273, 65274, 65275, 65535, 65536]
inputs = [text_corpus(rng, n) for n in sizes]
inputs += [paradise[i * 65536:(i + 1) * 65536] for i in range(3)]
inputs += [binary_corpus(rng, 65536), bytes(rng.getrandbits(8) for _ in range(65536)),
           b"a" * 65536, _periodic(rng, 65536), _overlay_stress(rng, 65536), bytes(65536),
           _periodic(rng, 40000) + bytes(rng.getrandbits(8) for _ in range(25536))]
os.makedirs("gpurun_out/dbg", exist_ok=True)
bad = 0
for level in range(4, 10):
    gpu = sdz.deflate_batch(inputs, level=level, format="raw")
    for i, (g, d) in enumerate(zip(gpu, inputs)):
        exp = O.deflate(d, level=level, format="raw")
        if g["data"] != exp:
            print("level", level, "input", i, len(d), "sizes", len(g["data"]), len(exp), g["status"])
            if bad < 4:
                open("gpurun_out/dbg/g%d_%d.bin" % (level, i), "wb").write(g["data"])
                open("gpurun_out/dbg/e%d_%d.bin" % (level, i), "wb").write(exp)
                open("gpurun_out/dbg/in%d_%d.bin" % (level, i), "wb").write(d)
            bad += 1
print("mismatches", bad)
