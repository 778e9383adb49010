/*
 * TypeScript declarations of the Node host shim (index.js): the observer subset of
 * @fluidframework/merge-tree's Client (packages/dds/merge-tree/src/client.ts:98) backed by the
 * MI355X engine through the N-API addon (mtr_napi.node) and the C ABI (include/mtr.h).
 */
import type { ISequencedDocumentMessage } from "@fluidframework/protocol-definitions";
import type { ISummaryTreeWithStats } from "@fluidframework/runtime-definitions";

/** IMergeTreeOptions subset (mergeTree.ts:400-438) plus engine capacities. */
export interface BatchReplayOptions {
	newLengthCalc?: 0 | 1; // mergeTreeUseNewLengthCalculations
	snapshotV1?: 0 | 1; // newMergeTreeSnapshotFormat
	chunkSize?: number; // mergeTreeSnapshotChunkSize (default 10000)
	catchUpBlobName?: string; // legacy catch-up blob name (default "catchupOps")
	device?: number; // HIP device ordinal
	maxSegments?: number;
	heapEntries?: number;
	textUnits?: number;
	propWords?: number;
	removerCells?: number;
	opsPerLaunch?: number;
}

/** Thrown for inputs outside the observer path: keep this document on the TypeScript Client. */
export class UnsupportedError extends Error {
	readonly fallback: true;
}

/** The observer Clients of many documents on one GPU; messages are applied in batches. */
export class BatchReplayEngine {
	constructor(maxDocs: number, options?: BatchReplayOptions);
	createClient(): BatchReplayClient;
	/** A SharedMatrix observer: its rows / cols PermutationVectors as two engine documents. */
	createMatrix(): BatchMatrixClient;
	/** Apply every queued message of every document (done implicitly before any read). */
	flush(): void;
	/** flush() on a libuv worker thread (napi_async_work); other calls on this engine throw until it settles. */
	flushAsync(): Promise<void>;
	/**
	 * The summarizer's hand-over in one call (mtr_replay_pipelined): apply every queued message, build every
	 * document's summary and download the records -- document d's is bytes[docOff[d], docOff[d + 1]): u32 blob
	 * count, u32 blob lengths, the blobs (the same bytes summarize() returns as blob contents).  Batches of remote
	 * messages go through the pipelined path in `parts` document ranges (pipelined: true); others take the serial
	 * calls.  The per-client summarize() reads stay valid afterwards.
	 */
	replaySummaries(parts?: number): { bytes: Buffer; docOff: Float64Array; pipelined: boolean };
}

/** getContainingSegment's answer (client.ts:1065-1078); both fields undefined when no segment covers pos. */
export interface ContainingSegment {
	segment?: {
		text?: string;
		marker?: { refType: number };
		cachedLength: number;
		seq: number;
		clientId: string; // the long id ("original" for the non-collaborating client)
		removedSeq?: number;
		leafIndex: number;
		propertySet?: number;
	};
	offset?: number;
}

/** SharedMatrix observer (matrix.ts:636-693, remote branch). */
export class BatchMatrixClient {
	startOrUpdateCollaboration(longClientId: string, minSeq?: number, currentSeq?: number): void;
	applyMsg(msg: ISequencedDocumentMessage): void;
	/** Each vector's PermutationVector.summarize blobs (V1 segments..., handleTable), permutationvector.ts:310-325. */
	summarizeVectors(): { rows: string[]; cols: string[] };
}

/** Drop-in for the observer use of `Client` (client.ts:98). */
export class BatchReplayClient {
	startOrUpdateCollaboration(longClientId: string, minSeq?: number, currentSeq?: number): void; // client.ts:1133
	applyMsg(msg: ISequencedDocumentMessage, local?: false): void; // client.ts:858
	updateSeqNumbers(min: number, seq: number): void; // client.ts:877
	insertTextLocal(pos: number, text: string, props?: Record<string, unknown>): void; // before collaboration only
	insertMarkerLocal(pos: number, refType: number, props?: Record<string, unknown>): void;
	removeRangeLocal(start: number, end: number): void;
	annotateRangeLocal(start: number, end: number, props: Record<string, unknown>): void;
	getText(): string; // MergeTreeTextHelper.getText, MergeTreeTextHelper.ts:20
	getLength(): number;
	getCurrentSeq(): number;
	/** interval collections (sequence/src/intervalCollection.ts): the summary's `header` blob before load ... */
	loadIntervals(header: string): void;
	/** ... and loadFinished (sequence.ts:750-801) after load and its catch-up messages */
	loadFinished(): void;
	/** a detached string's collection: add(start, end, intervalType, props with an intervalId) */
	getIntervalCollection(label: string): { add(start: number, end: number, intervalType: number, props: object): void };
	/** the summary's `header` blob (sequence.ts:467-480); undefined when there are no collections */
	summarizeIntervals(): string | undefined;
	summarize(
		runtime: { deltaManager: { minimumSequenceNumber: number; lastSequenceNumber: number } },
		handle: unknown,
		serializer: { stringify(value: unknown, bind: unknown): string } | undefined,
		catchUpMsgs: ISequencedDocumentMessage[],
	): ISummaryTreeWithStats; // client.ts:966
	/** summarize with the GPU work on a worker thread. */
	summarizeAsync(
		runtime: { deltaManager: { minimumSequenceNumber: number; lastSequenceNumber: number } },
		handle: unknown,
		serializer: { stringify(value: unknown, bind: unknown): string } | undefined,
		catchUpMsgs: ISequencedDocumentMessage[],
	): Promise<ISummaryTreeWithStats>;
	/** client.ts:1065: the segment holding pos at sequenceArgs' view (default: this client's current view). */
	getContainingSegment(
		pos: number,
		sequenceArgs?: { referenceSequenceNumber: number; clientId: string },
	): ContainingSegment;
}
