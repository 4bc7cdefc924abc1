// The reference's own perf case (test/perf.html:54-87) through the drop-in facade under Node:
// 20 samples each of deflate(paradiselost.txt, {level: 4}) and inflate(paradiselost.gz), the
// extremes dropped (perf.html:23-37), plus BASELINE C1, inflate(simple.deflate).  Prints one
// JSON line (ms).  Run on a GPU box: node tests/node/perf.mjs
import { readFileSync } from "fs";
import { fileURLToPath } from "url";
import { dirname, join } from "path";
import { performance } from "perf_hooks";
import { inflate, deflate } from "../../sd-zlib_amd/js/index.mjs";

const here = dirname(fileURLToPath(import.meta.url));
const golden = name => new Uint8Array(readFileSync(join(here, "..", "golden", name)));
const eq = (a, b) => a.length === b.length && a.every((v, i) => v === b[i]);

function calc(samp) {            // perf.html:23-37: sort, drop the min and the max, then the stats
	samp.sort((a, b) => a - b);
	samp.pop();
	samp.shift();
	const total = samp.reduce((s, t) => s + t, 0);
	return { count: samp.length, avg: +(total / samp.length).toFixed(3), min: +samp[0].toFixed(3),
		max: +samp[samp.length - 1].toFixed(3) };
}
function time(fn) {
	const t0 = performance.now();
	fn();
	return performance.now() - t0;
}

const text = golden("paradiselost.txt");
const gz = golden("paradiselost.gz");
const simple = golden("simple.deflate");
// parity of what is timed: L4 size from the reference's table, the gz round trip, C1
const ok = deflate(text, { level: 4 }).length === 203828 && eq(inflate(gz), text) &&
	eq(inflate(simple), golden("simple.txt"));
const defSamples = [], infSamples = [], c1Samples = [];
for (let k = 0; k < 20; ++k) {
	defSamples.push(time(() => deflate(text, { level: 4 })));
	infSamples.push(time(() => inflate(gz)));
	c1Samples.push(time(() => inflate(simple)));
}
console.log(JSON.stringify({
	deflate_L4_ms: calc(defSamples), inflate_gz_ms: calc(infSamples), inflate_simple_ms: calc(c1Samples),
	parity: ok, node: process.version,
	reference_browser_ms: { deflate_L4: "19-24", note: "test/perf.html:63-69 (L4 row); inflate has no published range" },
}));
