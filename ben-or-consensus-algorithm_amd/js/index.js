'use strict';
// JavaScript mirror of the reference's public surface, backed by the N-API
// addon (benor.node) over libbenor.so.  Drop-in for
//   src/index.ts:4-14            launchNetwork(N, F, initialValues, faultyList)
//   src/nodes/consensus.ts:3-15  startConsensus(N) / stopConsensus(N)
//   __test__/tests/utils.ts:4-24 getNodesState(N) / reachedFinality(states)
// plus what the HTTP routes served: getNodeState(i) (GET /getState,
// node.ts:197-199) and getNodeStatus(i) (GET /status, node.ts:33-39).
// As in the reference, one network "listens" at a time (ports 3000 + i there;
// the most recently launched network here).

const path = require('path');
const addon = require(path.join(__dirname, 'benor.node'));

const BASE_NODE_PORT = 3000;          // src/config.ts:1
const DEFAULT_K_MAX = 64;             // round cap: the reference runs until /stop

let current = null;                   // { handle, N }

// Stands in for the http.Server objects launchNetwork returns; the reference
// test teardown calls server.close(cb) and closeAllConnections()
// (benorconsensus.test.ts:14-29).
class NodeServer {
  constructor(nodeId) { this.nodeId = nodeId; this.port = BASE_NODE_PORT + nodeId; }
  close(cb) { if (typeof cb === 'function') setImmediate(cb); return this; }
  closeAllConnections() {}
}


// options.stopAfter -> an array of N entries (null = never stopped).  Keys
// must be node ids in [0, N): a bad key is a RangeError, not a launch error.
function stopSchedule(N, stopAfter) {
  if (Array.isArray(stopAfter) && stopAfter.length !== N)
    throw new RangeError(`stopAfter: an array must have N = ${N} entries, got ${stopAfter.length}`);
  const sched = new Array(N).fill(null);
  for (const [k, v] of Object.entries(stopAfter)) {
    const i = Number(k);
    if (!Number.isInteger(i) || i < 0 || i >= N) throw new RangeError(`stopAfter: node ${k} is not in [0, ${N})`);
    sched[i] = v;
  }
  return sched;
}

// The Value encoding of bo_network_create (0, 1, 2 = "?", anything else -2:
// rejected there) and launchNodes.ts:12's `el === true` for faulty nodes, done
// here so that the addon takes two typed arrays instead of 2N elements.
function encodeValues(initialValues) {
  const out = new Int8Array(initialValues.length);
  for (let i = 0; i < out.length; i++) {
    const v = initialValues[i];
    out[i] = v === 0 ? 0 : v === 1 ? 1 : v === '?' ? 2 : -2;
  }
  return out;
}

function encodeFaulty(faultyList) {
  const out = new Uint8Array(faultyList.length);
  for (let i = 0; i < out.length; i++) out[i] = faultyList[i] === true ? 1 : 0;
  return out;
}

async function launchNetwork(N, F, initialValues, faultyList) {
  // throws the reference's Errors (bo_network_create validates, in its order)
  const handle = Array.isArray(initialValues) && Array.isArray(faultyList)
    ? addon.networkCreateTyped(N, F, encodeValues(initialValues), encodeFaulty(faultyList))
    : addon.networkCreate(N, F, initialValues, faultyList);
  current = { handle, N, running: null };
  const servers = [];
  for (let i = 0; i < N; i++) servers.push(new NodeServer(i));
  return servers;
}

function net(N) {
  if (!current || (N !== undefined && current.N !== N)) throw new Error(`no launched network of size ${N}`);
  return current;
}

function randomSeed() {
  // the reference's coins come from Math.random(); a fresh 64-bit key per start
  const hi = BigInt(Math.floor(Math.random() * 2 ** 32));
  const lo = BigInt(Math.floor(Math.random() * 2 ** 32));
  return (hi << 32n) | lo;
}

// As the reference's (consensus.ts:3-8): resolves once every running node has
// served GET /start, i.e. as soon as the round loop is launched
// (bo_consensus_start_live), before consensus finishes (node.ts:167-188
// answers right after the round-1 broadcasts).  A stopConsensus / stopNode sent
// afterwards lands in the running kernel before its next delivery (node.ts:45,
// :191-194); getNodesState / getNodeState answer at once, as GET /getState does
// (node.ts:197-199), with a snapshot of the running network, so the reference's
// start-then-poll callers see the run progress and then its final states;
// waitConsensus(N) waits for the end.
// liveStopEvents(N) gives the delivery count at which each /stop landed
// (replayable as stopAfter on a fresh network with the same seed).
// options.sync: resolve when the round loop has run to completion (every live
// node decided, or kMax rounds); a /stop sent while it runs is ordered after it.
// options.stopAfter: GET /stop requests that land while consensus runs, given
// up front -- an array of N delivery counts or an object {nodeId: deliveries};
// a node is stopped after that many POST /message have been handled
// network-wide (seeded delivery order, the event-level kernel, N <= 4096).
// Resolves at the end of the run, like sync.
// A second start on the same network resolves, as the reference's GET /start
// answers 200, but runs nothing: its round inboxes outlive a run (node.ts:29-30),
// so no fresh consensus can follow (options.strict: reject with libbenor error 8).
async function startConsensus(N, options = {}) {
  if (N === 0) return;
  const seed = options.seed !== undefined ? BigInt(options.seed) : randomSeed();
  const kMax = options.kMax !== undefined ? options.kMax : DEFAULT_K_MAX;
  let sched;
  if (options.stopAfter !== undefined && options.stopAfter !== null) {
    if (options.live) throw new RangeError('stopAfter and live are exclusive: a live run takes /stop as it comes');
    sched = stopSchedule(N, options.stopAfter);
  }
  if (options.live && options.sync) throw new RangeError('live and sync are exclusive');
  // an explicit {live: false} is the run-to-completion form, as {sync: true}
  const live = sched === undefined && !options.sync && options.live !== false;
  const cur = net(N);
  try {
    if (live) {
      addon.networkStartLive(cur.handle, seed, kMax);
      // the end of the run, for waitConsensus / liveStopEvents (a failed run
      // also fails every later getNodeState / getNodesState, in libbenor)
      cur.running = addon.networkWait(cur.handle);
      cur.running.catch(() => {});
      return;
    }
    await addon.networkStart(cur.handle, seed, kMax, sched);
  } catch (e) {
    if (options.strict || !/libbenor error 8:/.test(e.message)) throw e;
  }
}

// The end of a live run (a no-op otherwise).  Concurrent readers all wait for
// the same run (the reference's getNodesState is Promise.all over
// getNodeState, __test__/tests/utils.ts:14-20).
async function settle(cur) {
  if (cur.running) await cur.running;
}

async function waitConsensus(N) {
  if (N === 0) return;
  await settle(net(N));
}

async function liveStopEvents(N) {
  const cur = net(N);
  await settle(cur);
  return addon.liveStopEvents(cur.handle);
}

async function stopConsensus(N) {
  if (N === 0) return;
  addon.networkStop(net(N).handle);
}

async function stopNode(nodeId) { addon.nodeStop(net().handle, nodeId); }

// GET /getState (node.ts:197-199): at once, the node's current state (a
// snapshot of a live run in flight; its final state once the run has ended).
async function getNodeState(nodeId) {
  return addon.getState(net().handle, nodeId);
}

// bo_node_state records (8 bytes: int8 killed, x, decided, pad; int32 k) ->
// NodeState objects (src/types.ts:1-8), as the addon's getState builds them.
function decodeStates(buf) {
  const b = new Int8Array(buf), k = new Int32Array(buf), n = b.length >> 3, out = new Array(n);
  for (let i = 0; i < n; i++) {
    const x = b[8 * i + 1], d = b[8 * i + 2], kk = k[2 * i + 1];
    out[i] = { killed: b[8 * i] !== 0, x: x < 0 ? null : x === 2 ? '?' : x, decided: d < 0 ? null : d !== 0,
               k: kk < 0 ? null : kk };
  }
  return out;
}

// __test__/tests/utils.ts:14-20: every node's state, from one snapshot.
async function getNodesState(N) {
  const cur = net(N);
  return decodeStates(addon.getStatesRaw(cur.handle).buf).slice(0, cur.N);
}

// The same with the delivery count a live run's snapshot reflects (null when
// no run is in flight): oracle (iii) truncated there gives the states.
async function getNodesStateAt(N) {
  const cur = net(N);
  const r = addon.getStatesRaw(cur.handle);
  return { states: decodeStates(r.buf).slice(0, cur.N), events: r.events };
}

// GET /status: { status: 500, body: "faulty" } | { status: 200, body: "live" }
async function getNodeStatus(nodeId) {
  const code = addon.status(net().handle, nodeId);
  return { status: code, body: code === 500 ? 'faulty' : 'live' };
}

function reachedFinality(states) {
  return states.find((el) => el.decided === false) === undefined;
}

// Batch of independent trials: resolves to the outcome histogram
// (BigUint64Array, layout documented in include/benor.h).
async function runTrials(cfg) { return addon.runTrials(cfg); }

const delay = (ms) => new Promise((res) => setTimeout(res, ms));   // src/utils.ts:1

module.exports = {
  BASE_NODE_PORT, DEFAULT_K_MAX, launchNetwork, startConsensus, stopConsensus, stopNode,
  getNodeState, getNodesState, getNodeStatus, reachedFinality, runTrials, delay,
  waitConsensus, liveStopEvents, getNodesStateAt,
};
