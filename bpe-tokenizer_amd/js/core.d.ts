// core.d.ts — type surface of the drop-in core.js; identical to beenotung/bpe-tokenizer v2.2.0
// core.ts (types core.ts:1-33, exports core.ts:36-75, class core.ts:77-495, compactMerge 500-503).
export type Token = {
  chars: string
  /** @description the weight after merge */
  weight: number
  /** @description the weight before merge */
  original_weight: number
  code: string
  /** @description including zero-weight tokens in token_table */
  index: number
}
export type MergeToken = [a: Token, b: Token, c: Token]
export type CompactMerge = [a_code: string, b_code: string, c_weight: number]
type MergeCode = [from_code: string, to_code: string]
export type BPETokenizerJSON = {
  version: 2
  char_count: number
  token_table: [chars: string, weight: number, original_weight: number][]
  merge_codes: [a_code: string, b_code: string, c_code: string][]
}
export declare let FS: string
export declare let EOF: string
export declare let LF: string
export declare let CR: string
export type Markers = {
  begin_marker: string
  end_marker: string
}
export declare function fileContentToCorpus(content: string | Buffer): string
export declare function linesToCorpus(text: string): string[]
export declare function linesTrimmedToCorpus(text: string): string[]
export declare class BPETokenizer {
  char_to_token: Record<string, Token>
  code_to_token: Record<string, Token>
  token_table: Token[]
  merge_tokens: MergeToken[]
  merge_codes: MergeCode[]
  to_vector_index: number[] | null
  from_vector_index: number[] | null
  /** materialised from HBM on read; assigning replaces the device corpus (`= []` clears it) */
  corpus_in_code: string[]
  toJSON(): BPETokenizerJSON
  fromJSON(json: BPETokenizerJSON): void
  protected invalidateVectorIndex(): void
  addToCorpus(content: string): void
  restoreToCorpus(content: string): void
  compactVectorIndex(): void
  findNextMerge(options?: { min_weight?: number; max_length?: number }): MergeToken | null
  applyMerge(merge: MergeToken): void
  mergeUntil(options?: { min_weight?: number; max_length?: number; max_iterations?: number }): void
  encodeToCode(content: string): string
  encodeToTokens(content: string): Token[]
  encodeToVector(content: string): number[]
  decodeTokens(tokens: Token[]): string
  decodeVector(vector: number[]): string
  restoreMerge(compactMerge: CompactMerge): void
}
export declare function compactMerge(merge: MergeToken): CompactMerge
export {}
