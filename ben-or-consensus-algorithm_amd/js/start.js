'use strict';
// node js/start.js -- the reference's `yarn start` scenario (src/start.ts:6-43)
// on the MI355X round loop: N = 10, nodes 0-3 faulty, every initial value 1;
// same checks ("Lengths don't match", "Too many faulty nodes" when more than
// half are faulty), then launchNetwork + startConsensus, then prints the
// nodes' states (the reference logs them from each node's handler instead).
//
// Optional: --N 10  --faulty 0,1,2,3  --init 1,1,...,?  --seed S  --kMax K
// (faultyArray has N entries, the ids listed in --faulty set; N defaults to the
// length of --init, so the two arrays can differ as in start.ts:7-21)
const benor = require('./index.js');

function arg(name) {
  const i = process.argv.indexOf(`--${name}`);
  return i >= 0 ? process.argv[i + 1] : undefined;
}

async function main() {
  const init = (arg('init') || '1,1,1,1,1,1,1,1,1,1').split(',').map((v) => (v === '?' ? '?' : Number(v)));
  const faultyIds = new Set((arg('faulty') || '0,1,2,3').split(',').filter((v) => v !== '').map(Number));
  const N = arg('N') !== undefined ? Number(arg('N')) : init.length;
  const faultyArray = Array.from({ length: N }, (_, i) => faultyIds.has(i));

  if (init.length !== faultyArray.length) throw new Error("Lengths don't match");            // start.ts:22-23
  if (faultyArray.filter((f) => f === true).length > init.length / 2)                        // start.ts:25-29
    throw new Error('Too many faulty nodes');

  await benor.launchNetwork(init.length, faultyArray.filter((el) => el === true).length, init, faultyArray);
  await benor.delay(200);                                                                     // start.ts:38
  const opts = {};
  if (arg('seed') !== undefined) opts.seed = BigInt(arg('seed'));
  if (arg('kMax') !== undefined) opts.kMax = Number(arg('kMax'));
  await benor.startConsensus(init.length, opts);                                              // start.ts:40
  const states = await benor.getNodesState(init.length);
  states.forEach((s, i) => console.log(`Node ${i}: ${JSON.stringify(s)}`));
}

main().catch((e) => {
  console.error(e.message);
  process.exit(1);
});
