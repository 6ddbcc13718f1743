// Type declarations for the JavaScript mirror (index.js).  The reference's
// types are src/types.ts:1-8; the signatures mirror src/index.ts:4-14 and
// src/nodes/consensus.ts:3-15.

export type Value = 0 | 1 | "?";

export type NodeState = {
  killed: boolean;
  x: Value | null;
  decided: boolean | null;
  k: number | null;
};

export declare const BASE_NODE_PORT: number;
export declare const DEFAULT_K_MAX: number;

/** Stand-in for the reference's http.Server per node. */
export interface NodeServer {
  readonly nodeId: number;
  readonly port: number;
  close(cb?: () => void): NodeServer;
  closeAllConnections(): void;
}

/** Rejects with Error("Arrays don't match") / Error("faultyList doesnt have F faulties"). */
export declare function launchNetwork(
  N: number,
  F: number,
  initialValues: Value[],
  faultyList: boolean[]
): Promise<NodeServer[]>;

export interface StartOptions {
  /** Philox key for the per-node coins (default: random, like Math.random()). */
  seed?: bigint | number;
  /** Round cap (default 64). */
  kMax?: number;
  /** GET /stop requests landing mid-run (node.ts:191-194): per node, the number of
   * POST /message deliveries (network-wide, seeded order) after which it is stopped;
   * an array of N entries (null = never) or {nodeId: deliveries}.  Event-level kernels,
   * N <= 4096.  Resolves at the end of the run. */
  stopAfter?: (number | null)[] | { [nodeId: number]: number };
  /** Reject a second start on one network (libbenor error 8) instead of resolving as a no-op. */
  strict?: boolean;
  /** Resolve once the run has finished (every live node decided, or kMax rounds); a stop
   * sent meanwhile is ordered after the run.  Default: resolve once the kernel is launched,
   * as the reference's startConsensus does (consensus.ts:3-8). */
  sync?: boolean;
  /** The default (launch, resolve, let stops land in the running kernel); exclusive with
   * stopAfter and sync. */
  live?: boolean;
}

/** Resolves once the round loop is launched (before consensus finishes, like GET /start);
 * stopNode / stopConsensus then land in the running kernel, getNodesState / getNodeState answer
 * at once with a snapshot of the running network (GET /getState, node.ts:197-199), and
 * waitConsensus waits for the end of the run.  {sync: true}: resolves after the run. */
export declare function startConsensus(N: number, options?: StartOptions): Promise<void>;
export declare function stopConsensus(N: number): Promise<void>;
export declare function stopNode(nodeId: number): Promise<void>;
export declare function getNodeState(nodeId: number): Promise<NodeState>;
export declare function getNodesState(N: number): Promise<NodeState[]>;
/** getNodesState with the delivery count a live run's snapshot reflects (null when no run is in
 * flight): the states are oracle (iii) truncated before that many POST /message deliveries. */
export declare function getNodesStateAt(N: number): Promise<{ states: NodeState[]; events: number | null }>;
export declare function getNodeStatus(nodeId: number): Promise<{ status: 200 | 500; body: "live" | "faulty" }>;
export declare function reachedFinality(states: NodeState[]): boolean;
export declare function delay(ms: number): Promise<void>;
/** End of a run started by the default startConsensus; resolves at once otherwise. */
export declare function waitConsensus(N: number): Promise<void>;
/** After a run started by the default startConsensus: per node, the delivery count at which its /stop landed (null = none);
 * as stopAfter on a fresh network with the same seed it reproduces the run. */
export declare function liveStopEvents(N: number): Promise<(number | null)[]>;

export interface TrialsConfig {
  N: number;
  F: number;
  /** default: the first F nodes are crash-faulty */
  faultyList?: boolean[];
  /** default: iid Bernoulli(1/2) per live node */
  initialValues?: Value[];
  seed?: bigint | number;
  kMax?: number;
  trialBegin?: bigint | number;
  trialCount?: bigint | number;
  /** 0 lockstep (default), 1 random delivery (f <= F), 2 event level (N <= 4096) */
  mode?: 0 | 1 | 2;
  /** event mode: deliveries after which node i is stopped (null = never) */
  crashAt?: (number | null)[];
  /** event mode, random schedule: stop crashCount live nodes at uniform delivery counts in [0, crashWindow) */
  crashCount?: number;
  crashWindow?: number;
}

/** Outcome histogram, (kMax + 1) * 3 + 1 bins (include/benor.h). */
export declare function runTrials(cfg: TrialsConfig): Promise<BigUint64Array>;
