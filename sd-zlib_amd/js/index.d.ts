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

export declare function inflateBatch(streams: BufferSource[], outCaps?: number[], format?: 0 | 1 | 2): InflateBatchRecord[];
export declare function deflateBatch(streams: BufferSource[],
	options?: { level?: number; format?: "raw" | "deflate" | "gzip"; mtime?: number }): { status: string; checksum: number; data: Uint8Array }[];
export declare function deviceCount(): number;
