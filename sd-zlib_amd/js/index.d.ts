// Type contract of the drop-in facade: the same exported names and signatures
// as @stardazed/zlib 1.0.1 (dist/sd-zlib.d.ts:11-149), plus the batched entry
// points of the MI355X engine.

export interface InflaterOptions {
	/** input has no zlib/gzip header or trailer (default false) */
	raw?: boolean;
	/** preset dictionary, used when a zlib stream sets FDICT */
	dictionary?: BufferSource;
}

export interface InflateResult {
	success: boolean;
	complete: boolean;
	checksum: "match" | "mismatch" | "unchecked";
	fileSize: "match" | "mismatch" | "unchecked";
	fileName: string;
	modDate: Date | undefined;
}

export declare class Inflater {
	constructor(options?: InflaterOptions);
	append(data: BufferSource): Uint8Array[];
	finish(): InflateResult;
}

export declare function inflate(data: BufferSource, dictionary?: BufferSource): Uint8Array;

export interface DeflaterOptions {
	format?: "raw" | "deflate" | "gzip";
	level?: number;
	dictionary?: BufferSource;
	fileName?: string;
}

export declare class Deflater {
	constructor(options?: DeflaterOptions);
	append(data: BufferSource): Uint8Array[];
	finish(): Uint8Array[];
}

export declare function deflate(data: BufferSource, options?: DeflaterOptions): Uint8Array;
export declare function mergeBuffers(buffers: Uint8Array[]): Uint8Array;
export declare function adler32(source: BufferSource, seed?: number): number;
export declare function crc32(source: BufferSource, seed?: number): number;

/** one record per stream of a batched GPU inflate */
export interface InflateBatchRecord {
	status: "OK" | "DATA_ERROR" | "NEED_DICT" | "DICT_MISMATCH" | "TRUNCATED" | "OUT_OVERFLOW" |
		"TRAILING" | "TOO_SMALL" | "BAD_RECORD";
	zmsg: string;
	complete: boolean;
	success: boolean;
	checksum: "match" | "mismatch" | "unchecked";
	fileSize: "match" | "mismatch" | "unchecked";
	fileName: string;
	mtime: number;
	container: number;
	data: Uint8Array;
}

/** Multi-GPU stats (sdz_multi_stats): present on the result array when `devices` was given. */
export interface MultiStats {
	wallMs: number;
	computeMs: number;
	/** record all-gather, timed apart from compute */
	gatherMs: number;
	/** true: ncclAllGather over distinct devices; false: loopback (a device listed twice) */
	rccl: boolean;
	/** one entry per device of the list, in list order (LPT shards) */
	shards: { streams: number; bytesIn: number; bytesOut: number; kernelMs: number }[];
}

export interface InflateBatchOptions {
	/** output slot per stream (default max(64 KiB, 8 x input)) */
	outCaps?: number[];
	/** 0 raw, 1 zlib/gzip, 2 auto-detect as inflate() (default 2) */
	format?: 0 | 1 | 2;
	dictionary?: BufferSource;
	/** GPUs to shard over (LPT by size, one host thread per GPU, records gathered over RCCL) */
	devices?: number[];
}
export interface DeflateBatchOptions {
	level?: number;
	format?: "raw" | "deflate" | "gzip";
	fileName?: string;
	mtime?: number;
	dictionary?: BufferSource;
	devices?: number[];
}

export declare function inflateBatch(streams: BufferSource[], options?: InflateBatchOptions | number[],
	format?: 0 | 1 | 2): InflateBatchRecord[] & { stats?: MultiStats };
export declare function deflateBatch(streams: BufferSource[], options?: DeflateBatchOptions):
	{ status: string; checksum: number; data: Uint8Array }[] & { stats?: MultiStats };
export declare function deviceCount(): number;
