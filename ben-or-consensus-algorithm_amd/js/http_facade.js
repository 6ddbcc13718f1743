'use strict';
// HTTP facade: the reference's per-node routes, wire-compatible, served from
// the simulated network state (SURVEY §8f #1).  With it, the reference's
// src/nodes/consensus.ts (fetch GET /start, /stop on 3000 + i) and
// __test__/tests/utils.ts (fetch GET /getState) work unchanged; only
// src/index.ts's launchNetwork is swapped for the one below.
//
// Routes per node i on port basePort + i (node.ts:33-199):
//   GET  /status    500 "faulty" | 200 "live"                    node.ts:33-39
//   GET  /getState  200 NodeState JSON                           node.ts:197-199
//   GET  /start     200 {"message":"Algorithm started"}          node.ts:167-188
//   GET  /stop      200 "killed"                                 node.ts:191-194
//   POST /message   200 {"message":"Message received"}           node.ts:43-163
// The round loop itself runs on the GPU (one kernel launch) once every running
// node has received /start -- the point at which, in the reference, all live
// nodes have broadcast their round-1 proposals.  Until then a started node
// reports k = 1 (node.ts:172).  Messages POSTed from outside are acknowledged
// and not simulated (why: DESIGN.md §2); as in the reference (node.ts:45,161), a killed node
// never answers /message (the request stays open until the server closes).
// The round loop runs once per network: the reference's round inboxes
// (node.ts:29-30) outlive a run, so a later /start is acknowledged as the
// reference acknowledges it but starts no second run (bo_consensus_start
// refuses a second start on a network, include/benor.h).
const http = require('http');
const path = require('path');
const addon = require(path.join(__dirname, 'benor.node'));

const BASE_NODE_PORT = 3000;   // src/config.ts:1


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

async function launchNetwork(N, F, initialValues, faultyList, options = {}) {
  const basePort = options.basePort !== undefined ? options.basePort : BASE_NODE_PORT;
  const kMax = options.kMax !== undefined ? options.kMax : 64;
  // The run starts when every running node has served /start, and /start
  // answers at once (node.ts:167-188 answers before consensus finishes); a
  // GET /stop served over HTTP while it runs lands in the kernel
  // (bo_consensus_start_live), and /getState answers at once with a snapshot
  // of the running network, then its final states -- the reference's callers
  // poll it.
  // options.sync: /start answers once the run has finished; a /stop arriving
  // over HTTP while it is in flight is ordered after it.
  // options.stopAfter: GET /stop requests that land during the run, as delivery
  // counts per node (array of N, null = never; bo_consensus_start_sched), given
  // up front; /start answers at the end of the run, as with sync.
  let sched;
  if (options.stopAfter !== undefined && options.stopAfter !== null) {
    if (options.live) throw new RangeError('stopAfter and live are exclusive: a live run takes /stop as it comes');
    sched = stopSchedule(N, options.stopAfter);
  }
  if (options.live && options.sync) throw new RangeError('live and sync are exclusive');
  // an explicit {live: false} is the run-to-completion form, as {sync: true}
  const live = sched === undefined && !options.sync && options.live !== false;
  const handle = addon.networkCreate(N, F, initialValues, faultyList);   // launchNodes.ts:10-13 errors
  const net = {
    handle, N, started: new Array(N).fill(false), running: null, ran: false, seed: options.seed,
  };

  const runningNodes = () => {
    const r = [];
    for (let i = 0; i < N; i++) if (addon.status(handle, i) !== 500) r.push(i);
    return r;
  };

  function maybeRun() {
    if (net.running || net.ran) return live ? null : net.running;
    const run = runningNodes();
    if (run.length === 0 || !run.every((i) => net.started[i])) return null;
    let seed = net.seed;
    if (seed === undefined) {
      seed = (BigInt(Math.floor(Math.random() * 2 ** 32)) << 32n) | BigInt(Math.floor(Math.random() * 2 ** 32));
    }
    const done = () => {
      net.ran = true;
      net.running = null;
    };
    if (live) {
      try {
        addon.networkStartLive(handle, BigInt(seed), kMax);
      } catch (e) {
        return Promise.reject(e);
      }
      net.running = addon.networkWait(handle).then(done);
      net.running.catch(() => {});
      return Promise.resolve();   // launched: /start answers now
    }
    net.running = addon.networkStart(handle, BigInt(seed), kMax, sched).then(done);
    return net.running;
  }

  // GET /getState (node.ts:197-199) answers at once: a live run in flight
  // serves a snapshot of the running kernel (bo_get_state)
  function state(i) {
    const s = addon.getState(handle, i);
    if (!net.ran && !(live && net.running) && net.started[i] && !s.killed) s.k = 1;   // node.ts:172, before the run lands
    return s;
  }

  function send(res, code, body, json) {
    const data = json ? JSON.stringify(body) : String(body);
    res.writeHead(code, { 'Content-Type': json ? 'application/json; charset=utf-8' : 'text/html; charset=utf-8' });
    res.end(data);
  }

  function handler(i) {
    return (req, res) => {
      const url = req.url.split('?')[0];
      if (req.method === 'GET' && url === '/status') {
        return addon.status(handle, i) === 500 ? send(res, 500, 'faulty') : send(res, 200, 'live');
      }
      if (req.method === 'GET' && url === '/getState') return send(res, 200, state(i), true);
      if (req.method === 'GET' && url === '/stop') {
        addon.nodeStop(handle, i);
        return send(res, 200, 'killed');
      }
      if (req.method === 'GET' && url === '/start') {
        if (addon.status(handle, i) !== 500) net.started[i] = true;
        const p = maybeRun();
        const reply = () => send(res, 200, { message: 'Algorithm started' }, true);
        // respond once the round loop is launched (live), or has run (sync)
        if (p) p.then(reply, (e) => send(res, 500, { message: String(e && e.message) }, true));
        else reply();
        return undefined;
      }
      if (req.method === 'POST' && url === '/message') {
        req.resume();
        if (addon.status(handle, i) === 500) return undefined;   // node.ts:45,161: no reply
        return send(res, 200, { message: 'Message received' }, true);
      }
      return send(res, 404, 'not found');
    };
  }

  const servers = [];
  await Promise.all(Array.from({ length: N }, (_, i) => new Promise((resolve, reject) => {
    const srv = http.createServer(handler(i));
    srv.on('error', reject);
    srv.listen(basePort + i, () => resolve());
    servers[i] = srv;
  })));
  return servers;
}

module.exports = { BASE_NODE_PORT, launchNetwork };
