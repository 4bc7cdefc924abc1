// Node smoke test of the drop-in facade, modelled on the reference's test/index.html
// cases (inflate text/gzip/raw/parts/binary, gzip round trip).  Runs on a GPU box:
//   node tests/node/smoke.mjs
import { readFileSync } from "fs";
import { fileURLToPath } from "url";
import { dirname, join } from "path";
import { inflate, deflate, Inflater, Deflater, adler32, crc32, mergeBuffers, inflateBatch, deflateBatch } from "../../sd-zlib_amd/js/index.mjs";

const here = dirname(fileURLToPath(import.meta.url));
const golden = name => new Uint8Array(readFileSync(join(here, "..", "golden", name)));
const eq = (a, b) => a.length === b.length && a.every((v, i) => v === b[i]);
let failures = 0;
function check(name, cond) {
	console.log((cond ? "ok   " : "FAIL ") + name);
	if (!cond) failures++;
}

const text = golden("paradiselost.txt");
check("inflate(simple.deflate)", eq(inflate(golden("simple.deflate")), golden("simple.txt")));
check("inflate(paradiselost.deflate)", eq(inflate(golden("paradiselost.deflate")), text));
check("inflate(simple.raw) auto-detect", eq(inflate(golden("simple.raw")), golden("simple.txt")));
{
	const inf = new Inflater();
	const out = mergeBuffers(inf.append(golden("paradiselost.gz")));
	const res = inf.finish();
	check("Inflater gzip + verdicts", eq(out, text) && res.success && res.checksum === "match" &&
		res.fileSize === "match" && res.fileName === "paradiselost.txt" && res.modDate instanceof Date);
}
{
	const inf = new Inflater();
	const a = inf.append(golden("paradiselost.part1.deflate"));
	const b = inf.append(golden("paradiselost.part2.deflate"));
	check("Inflater two parts", eq(mergeBuffers(a.concat(b)), text) && inf.finish().success);
}
{
	// every header, block header and symbol crossing appends: 1..5-byte pieces
	const gz = golden("simple.gz");
	const inf = new Inflater();
	const parts = [];
	for (let i = 0, k = 1; i < gz.length; i += k, k = k % 5 + 1) parts.push(...inf.append(gz.subarray(i, i + k)));
	const res = inf.finish();
	check("Inflater gzip in 1..5-byte pieces", eq(mergeBuffers(parts), golden("simple.txt")) && res.success &&
		res.fileName === "simple.txt");
	let msg = "";
	try { inf.append(new Uint8Array([1, 2])); } catch (e) { msg = e.message; }
	check("append after the end: bad input data", msg === "inflate error: bad input data");
}
{
	const inf = new Inflater();
	inf.append(golden("vertices.deflate"));
	check("Inflater binary (vertices)", inf.finish().checksum === "match");
}
{
	const d = new Deflater({ level: 6, format: "gzip", fileName: "paradiselost.orig" });
	const comp = mergeBuffers(d.append(text).concat(d.finish()));
	const inf = new Inflater();
	const out = mergeBuffers(inf.append(comp));
	check("gzip round trip", eq(out, text) && inf.finish().fileName === "paradiselost.orig");
}
check("deflate L6 == reference fixture", eq(deflate(text, { level: 6 }), golden("paradiselost.deflate")));
{
	// Deflater.append in pieces: output arrives per append (complete blocks), and the merged
	// stream is the reference's
	const d = new Deflater({ level: 6 });
	const outs = [];
	for (let i = 0, k = 1; i < text.length; i += k, k = k * 3 % 70001 + 1) outs.push(...d.append(text.subarray(i, i + k)));
	const early = mergeBuffers(outs).length;
	outs.push(...d.finish());
	check("Deflater in pieces == reference fixture", eq(mergeBuffers(outs), golden("paradiselost.deflate")) && early > 100000);
	let m = "";
	try { new Deflater().finish(); } catch (e) { m = e.message; }
	check("finish before append", m === "Cannot call finish before at least 1 call to append");
}
{
	// test/index.html:173-208: a preset dictionary round trip ("deflate" container)
	const words = new TextEncoder().encode("the of and to in that with his her for thou thy thee");
	const src = text.subarray(2000, 30000);
	const comp = deflate(src, { level: 6, dictionary: words });
	const inf = new Inflater({ dictionary: words });
	const out = mergeBuffers(inf.append(comp));
	check("dictionary round trip", comp[0] === 0x78 && comp[1] === 0x20 && eq(out, src) && inf.finish().success);
}
{
	// the reference's arrays: Inflater.append -> 16 KiB ZStream passes (sd-inflate.ts:101-150)
	const inf = new Inflater();
	const a = inf.append(golden("paradiselost.part1.deflate"));
	const b = inf.append(golden("paradiselost.part2.deflate"));
	const full = x => x.slice(0, -1).every(c => c.length === 16384);
	check("Inflater arrays are 16 KiB passes", a.length > 1 && b.length > 1 && full(a) && full(b) &&
		eq(mergeBuffers(a.concat(b)), text));
	// Deflater: the header alone, 16 KiB passes, the trailer alone (sd-deflate.ts:199-250)
	const d = new Deflater({ level: 6, format: "gzip", fileName: "p.txt" });
	const x = d.append(text);
	const f = d.finish();
	check("Deflater arrays: header | passes | trailer", x[0].length === 10 + 6 && full(x.slice(1)) &&
		f[f.length - 1].length === 8 && full(f.slice(0, -1)));
	let m = "";
	try { d.append(new Uint8Array([1, 2, 3])); } catch (e) { m = e.message; }
	check("append after finish: deflating + z.msg", m === "deflating: ");
}
{
	// a gzip FNAME longer than 64 KiB comes back whole
	const name = "n".repeat(70000) + ".txt";
	const d = new Deflater({ level: 6, format: "gzip", fileName: name });
	const comp = mergeBuffers(d.append(golden("simple.txt")).concat(d.finish()));
	const inf = new Inflater();
	inf.append(comp);
	check("gzip FNAME > 64 KiB", inf.finish().fileName === name);
}
{
	// batched entry points over GPUs: LPT shards, records all-gathered (RCCL one rank / loopback)
	const streams = [golden("paradiselost.deflate"), golden("simple.deflate"), golden("paradiselost.gz"),
		golden("simple.raw")];
	const want = [text, golden("simple.txt"), text, golden("simple.txt")];
	for (const devices of [[0], [0, 0]]) {
		const r = inflateBatch(streams, { outCaps: want.map(w => w.length + 64), devices });
		check("inflateBatch devices " + JSON.stringify(devices), r.every((x, i) => x.success && eq(x.data, want[i])) &&
			r.stats && r.stats.shards.length === devices.length && r.stats.rccl === (devices.length === 1));
	}
	const dz = deflateBatch([text, golden("simple.txt")], { level: 6, devices: [0, 0] });
	check("deflateBatch devices [0,0]", eq(dz[0].data, golden("paradiselost.deflate")) &&
		eq(dz[1].data, golden("simple.deflate")));
}
{
	// inflate()'s errors (one-shot path) are the ones an Inflater append + finish gives
	const s = golden("simple.deflate");
	const viaInflater = data => {
		const inf = new Inflater();
		try { inf.append(data); } catch (e) { return e.message; }
		const r = inf.finish();
		return r.success ? "" : !r.complete ? "Unexpected EOF during decompression" :
			r.checksum === "mismatch" ? "Data integrity check failed" : "Decompression error";
	};
	const bad = s.slice();
	bad[bad.length - 1] ^= 1;
	const junk = s.slice();
	junk[2] = 0xff;
	for (const [name, data] of [["truncated", s.subarray(0, s.length - 6)], ["bad adler32", bad], ["bad block", junk]]) {
		let m = "";
		try { inflate(data); } catch (e) { m = e.message; }
		check("inflate " + name + ": " + m, m !== "" && m === viaInflater(data));
	}
	// a stream that expands ~1000x overflows the one-shot slot: inflate() takes the Inflater path, with
	// the same bytes, and the same error for a corrupted copy
	const zeros = new Uint8Array(1 << 20);
	const zc = deflate(zeros, { level: 9 });
	check("inflate 1 MiB of zeros (" + zc.length + " B in)", eq(inflate(zc), zeros));
	const zbad = zc.slice();
	zbad[zbad.length - 1] ^= 1;
	let zm = "";
	try { inflate(zbad); } catch (e) { zm = e.message; }
	check("inflate zeros, bad adler32: " + zm, zm !== "" && zm === viaInflater(zbad));
}
check("adler32 KAT", adler32(golden("simple.txt")) === -1612443532);
check("crc32 KAT", crc32(golden("simple.txt")) === 1488305224);
let threw = "";
try { inflate(new Uint8Array([1])); } catch (e) { threw = e.message; }
check("error message: too small", threw === "data buffer is too small");
threw = "";
try { new Deflater({ level: 10 }); } catch (e) { threw = e.constructor.name + ":" + e.message; }
check("RangeError level", threw === "RangeError:level must be between 1 and 9, inclusive");
process.exit(failures ? 1 : 0);
