// poseidon.h — Poseidon-Goldilocks permutation for the MI355X prover.
// Width 12, rate 8, S-box x^7, 4 + 22 + 4 rounds, MDS circulant
// [17,15,41,16,2,28,13,13,39,18,34,20] + diag [8,0..0].
// Replaces qp-plonky2 1.1.1 hash/poseidon.rs + poseidon_goldilocks.rs.
// Round constants: plonky2 ALL_ROUND_CONSTANTS (SURVEY.md Appendix C,
// SHA-256 d2fcbb5b...a8 over the 360 LE u64, checked in tests/test_abi.py).
//
// Device form: the state lives in 12 u64 VGPR pairs; the MDS layer uses the
// small constants via 32x32->64 multiply-accumulates of the split state
// (no 64x64 products), one reduction per output lane.
#pragma once
#include "field.h"

namespace ps {

constexpr int WIDTH = 12, RATE = 8, ROUNDS = 30, HALF_FULL = 4, PARTIAL = 22;

__host__ __device__ constexpr uint32_t mds_circ(int i) {
  return i == 0 ? 17 : i == 1 ? 15 : i == 2 ? 41 : i == 3 ? 16 : i == 4 ? 2 : i == 5 ? 28 : i == 6 ? 13
       : i == 7 ? 13 : i == 8 ? 39 : i == 9 ? 18 : i == 10 ? 34 : 20;
}

#define QP_POSEIDON_RC_LIST \
    0xb585f766f2144405ULL, 0x7746a55f43921ad7ULL, 0xb2fb0d31cee799b4ULL, 0x0f6760a4803427d7ULL, \
    0xe10d666650f4e012ULL, 0x8cae14cb07d09bf1ULL, 0xd438539c95f63e9fULL, 0xef781c7ce35b4c3dULL, \
    0xcdc4a239b0c44426ULL, 0x277fa208bf337bffULL, 0xe17653a29da578a1ULL, 0xc54302f225db2c76ULL, \
    0x86287821f722c881ULL, 0x59cd1a8a41c18e55ULL, 0xc3b919ad495dc574ULL, 0xa484c4c5ef6a0781ULL, \
    0x308bbd23dc5416ccULL, 0x6e4a40c18f30c09cULL, 0x9a2eedb70d8f8cfaULL, 0xe360c6e0ae486f38ULL, \
    0xd5c7718fbfc647fbULL, 0xc35eae071903ff0bULL, 0x849c2656969c4be7ULL, 0xc0572c8c08cbbbadULL, \
    0xe9fa634a21de0082ULL, 0xf56f6d48959a600dULL, 0xf7d713e806391165ULL, 0x8297132b32825dafULL, \
    0xad6805e0e30b2c8aULL, 0xac51d9f5fcf8535eULL, 0x502ad7dc18c2ad87ULL, 0x57a1550c110b3041ULL, \
    0x66bbd30e6ce0e583ULL, 0x0da2abef589d644eULL, 0xf061274fdb150d61ULL, 0x28b8ec3ae9c29633ULL, \
    0x92a756e67e2b9413ULL, 0x70e741ebfee96586ULL, 0x019d5ee2af82ec1cULL, 0x6f6f2ed772466352ULL, \
    0x7cf416cfe7e14ca1ULL, 0x61df517b86a46439ULL, 0x85dc499b11d77b75ULL, 0x4b959b48b9c10733ULL, \
    0xe8be3e5da8043e57ULL, 0xf5c0bc1de6da8699ULL, 0x40b12cbf09ef74bfULL, 0xa637093ecb2ad631ULL, \
    0x3cc3f892184df408ULL, 0x2e479dc157bf31bbULL, 0x6f49de07a6234346ULL, 0x213ce7bede378d7bULL, \
    0x5b0431345d4dea83ULL, 0xa2de45780344d6a1ULL, 0x7103aaf94a7bf308ULL, 0x5326fc0d97279301ULL, \
    0xa9ceb74fec024747ULL, 0x27f8ec88bb21b1a3ULL, 0xfceb4fda1ded0893ULL, 0xfac6ff1346a41675ULL, \
    0x7131aa45268d7d8cULL, 0x9351036095630f9fULL, 0xad535b24afc26bfbULL, 0x4627f5c6993e44beULL, \
    0x645cf794b8f1cc58ULL, 0x241c70ed0af61617ULL, 0xacb8e076647905f1ULL, 0x3737e9db4c4f474dULL, \
    0xe7ea5e33e75fffb6ULL, 0x90dee49fc9bfc23aULL, 0xd1b1edf76bc09c92ULL, 0x0b65481ba645c602ULL, \
    0x99ad1aab0814283bULL, 0x438a7c91d416ca4dULL, 0xb60de3bcc5ea751cULL, 0xc99cab6aef6f58bcULL, \
    0x69a5ed92a72ee4ffULL, 0x5e7b329c1ed4ad71ULL, 0x5fc0ac0800144885ULL, 0x32db829239774ecaULL, \
    0x0ade699c5830f310ULL, 0x7cc5583b10415f21ULL, 0x85df9ed2e166d64fULL, 0x6604df4fee32bcb1ULL, \
    0xeb84f608da56ef48ULL, 0xda608834c40e603dULL, 0x8f97fe408061f183ULL, 0xa93f485c96f37b89ULL, \
    0x6704e8ee8f18d563ULL, 0xcee3e9ac1e072119ULL, 0x510d0e65e2b470c1ULL, 0xf6323f486b9038f0ULL, \
    0x0b508cdeffa5ceefULL, 0xf2417089e4fb3cbdULL, 0x60e75c2890d15730ULL, 0xa6217d8bf660f29cULL, \
    0x7159cd30c3ac118eULL, 0x839b4e8fafead540ULL, 0x0d3f3e5e82920adcULL, 0x8f7d83bddee7bba8ULL, \
    0x780f2243ea071d06ULL, 0xeb915845f3de1634ULL, 0xd19e120d26b6f386ULL, 0x016ee53a7e5fecc6ULL, \
    0xcb5fd54e7933e477ULL, 0xacb8417879fd449fULL, 0x9c22190be7f74732ULL, 0x5d693c1ba3ba3621ULL, \
    0xdcef0797c2b69ec7ULL, 0x3d639263da827b13ULL, 0xe273fd971bc8d0e7ULL, 0x418f02702d227ed5ULL, \
    0x8c25fda3b503038cULL, 0x2cbaed4daec8c07cULL, 0x5f58e6afcdd6ddc2ULL, 0x284650ac5e1b0ebaULL, \
    0x635b337ee819dab5ULL, 0x9f9a036ed4f2d49fULL, 0xb93e260cae5c170eULL, 0xb0a7eae879ddb76dULL, \
    0xd0762cbc8ca6570cULL, 0x34c6efb812b04bf5ULL, 0x40bf0ab5fa14c112ULL, 0xb6b570fc7c5740d3ULL, \
    0x5a27b9002de33454ULL, 0xb1a5b165b6d2b2d2ULL, 0x8722e0ace9d1be22ULL, 0x788ee3b37e5680fbULL, \
    0x14a726661551e284ULL, 0x98b7672f9ef3b419ULL, 0xbb93ae776bb30e3aULL, 0x28fd3b046380f850ULL, \
    0x30a4680593258387ULL, 0x337dc00c61bd9ce1ULL, 0xd5eca244c7a4ff1dULL, 0x7762638264d279bdULL, \
    0xc1e434bedeefd767ULL, 0x0299351a53b8ec22ULL, 0xb2d456e4ad251b80ULL, 0x3e9ed1fda49cea0bULL, \
    0x2972a92ba450bed8ULL, 0x20216dd77be493deULL, 0xadffe8cf28449ec6ULL, 0x1c4dbb1c4c27d243ULL, \
    0x15a16a8a8322d458ULL, 0x388a128b7fd9a609ULL, 0x2300e5d6baedf0fbULL, 0x2f63aa8647e15104ULL, \
    0xf1c36ce86ecec269ULL, 0x27181125183970c9ULL, 0xe584029370dca96dULL, 0x4d9bbc3e02f1cfb2ULL, \
    0xea35bc29692af6f8ULL, 0x18e21b4beabb4137ULL, 0x1e3b9fc625b554f4ULL, 0x25d64362697828fdULL, \
    0x5a3f1bb1c53a9645ULL, 0xdb7f023869fb8d38ULL, 0xb462065911d4e1fcULL, 0x49c24ae4437d8030ULL, \
    0xd793862c112b0566ULL, 0xaadd1106730d8febULL, 0xc43b6e0e97b0d568ULL, 0xe29024c18ee6fca2ULL, \
    0x5e50c27535b88c66ULL, 0x10383f20a4ff9a87ULL, 0x38e8ee9d71a45af8ULL, 0xdd5118375bf1a9b9ULL, \
    0x775005982d74d7f7ULL, 0x86ab99b4dde6c8b0ULL, 0xb1204f603f51c080ULL, 0xef61ac8470250ecfULL, \
    0x1bbcd90f132c603fULL, 0x0cd1dabd964db557ULL, 0x11a3ae5beb9d1ec9ULL, 0xf755bfeea585d11dULL, \
    0xa3b83250268ea4d7ULL, 0x516306f4927c93afULL, 0xddb4ac49c9efa1daULL, 0x64bb6dec369d4418ULL, \
    0xf9cc95c22b4c1fccULL, 0x08d37f755f4ae9f6ULL, 0xeec49b613478675bULL, 0xf143933aed25e0b0ULL, \
    0xe4c5dd8255dfc622ULL, 0xe7ad7756f193198eULL, 0x92c2318b87fff9cbULL, 0x739c25f8fd73596dULL, \
    0x5636cac9f16dfed0ULL, 0xdd8f909a938e0172ULL, 0xc6401fe115063f5bULL, 0x8ad97b33f1ac1455ULL, \
    0x0c49366bb25e8513ULL, 0x0784d3d2f1698309ULL, 0x530fb67ea1809a81ULL, 0x410492299bb01f49ULL, \
    0x139542347424b9acULL, 0x9cb0bd5ea1a1115eULL, 0x02e3f615c38f49a1ULL, 0x985d4f4a9c5291efULL, \
    0x775b9feafdcd26e7ULL, 0x304265a6384f0f2dULL, 0x593664c39773012cULL, 0x4f0a2e5fb028f2ceULL, \
    0xdd611f1000c17442ULL, 0xd8185f9adfea4fd0ULL, 0xef87139ca9a3ab1eULL, 0x3ba71336c34ee133ULL, \
    0x7d3a455d56b70238ULL, 0x660d32e130182684ULL, 0x297a863f48cd1f43ULL, 0x90e0a736a751ebb7ULL, \
    0x549f80ce550c4fd3ULL, 0x0f73b2922f38bd64ULL, 0x16bf1f73fb7a9c3fULL, 0x6d1f5a59005bec17ULL, \
    0x02ff876fa5ef97c4ULL, 0xc5cb72a2a51159b0ULL, 0x8470f39d2d5c900eULL, 0x25abb3f1d39fcb76ULL, \
    0x23eb8cc9b372442fULL, 0xd687ba55c64f6364ULL, 0xda8d9e90fd8ff158ULL, 0xe3cbdc7d2fe45ea7ULL, \
    0xb9a8c9b3aee52297ULL, 0xc0d28a5c10960bd3ULL, 0x45d7ac9b68f71a34ULL, 0xeeb76e397069e804ULL, \
    0x3d06c8bd1514e2d9ULL, 0x9c9c98207cb10767ULL, 0x65700b51aedfb5efULL, 0x911f451539869408ULL, \
    0x7ae6849fbc3a0ec6ULL, 0x3bb340eba06afe7eULL, 0xb46e9d8b682ea65eULL, 0x8dcf22f9a3b34356ULL, \
    0x77bdaeda586257a7ULL, 0xf19e400a5104d20dULL, 0xc368a348e46d950fULL, 0x9ef1cd60e679f284ULL, \
    0xe89cd854d5d01d33ULL, 0x5cd377dc8bb882a2ULL, 0xa7b0fb7883eee860ULL, 0x7684403ec392950dULL, \
    0x5fa3f06f4fed3b52ULL, 0x8df57ac11bc04831ULL, 0x2db01efa1e1e1897ULL, 0x54846de4aadb9ca2ULL, \
    0xba6745385893c784ULL, 0x541d496344d2c75bULL, 0xe909678474e687feULL, 0xdfe89923f6c9c2ffULL, \
    0xece5a71e0cfedc75ULL, 0x5ff98fd5d51fe610ULL, 0x83e8941918964615ULL, 0x5922040b47f150c1ULL, \
    0xf97d750e3dd94521ULL, 0x5080d4c2b86f56d7ULL, 0xa7de115b56c78d70ULL, 0x6a9242ac87538194ULL, \
    0xf7856ef7f9173e44ULL, 0x2265fc92feb0dc09ULL, 0x17dfc8e4f7ba8a57ULL, 0x9001a64209f21db8ULL, \
    0x90004c1371b893c5ULL, 0xb932b7cf752e5545ULL, 0xa0b1df81b6fe59fcULL, 0x8ef1dd26770af2c2ULL, \
    0x0541a4f9cfbeed35ULL, 0x9e61106178bfc530ULL, 0xb3767e80935d8af2ULL, 0x0098d5782065af06ULL, \
    0x31d191cd5c1466c7ULL, 0x410fefafa319ac9dULL, 0xbdf8f242e316c4abULL, 0x9e8cd55b57637ed0ULL, \
    0xde122bebe9a39368ULL, 0x4d001fd58f002526ULL, 0xca6637000eb4a9f8ULL, 0x2f2339d624f91f78ULL, \
    0x6d1a7918c80df518ULL, 0xdf9a4939342308e9ULL, 0xebc2151ee6c8398cULL, 0x03cc2ba8a1116515ULL, \
    0xd341d037e840cf83ULL, 0x387cb5d25af4afccULL, 0xbba2515f22909e87ULL, 0x7248fe7705f38e47ULL, \
    0x4d61e56a525d225aULL, 0x262e963c8da05d3dULL, 0x59e89b094d220ec2ULL, 0x055d5b52b78b9c5eULL, \
    0x82b27eb33514ef99ULL, 0xd30094ca96b7ce7bULL, 0xcf5cb381cd0a1535ULL, 0xfeed4db6919e5a7cULL, \
    0x41703f53753be59fULL, 0x5eeea940fcde8b6fULL, 0x4cd1f1b175100206ULL, 0x4a20358574454ec0ULL, \
    0x1478d361dbbf9facULL, 0x6f02dc07d141875cULL, 0x296a202ed8e556a2ULL, 0x2afd67999bf32ee5ULL, \
    0x7acfd96efa95491dULL, 0x6798ba0c0abb2c6dULL, 0x34c6f57b26c92122ULL, 0x5736e1bad206b5deULL, \
    0x20057d2a0056521bULL, 0x3dea5bd5d0578bd7ULL, 0x16e50d897d4634acULL, 0x29bff3ecb9b7a6e3ULL, \
    0x475cd3205a3bdcdeULL, 0x18a42105c31b7e88ULL, 0x023e7414af663068ULL, 0x15147108121967d7ULL, \
    0xe4a3dff1d7d6fef9ULL, 0x01a8d1a588085737ULL, 0x11b4c74eda62beefULL, 0xe587cc0d69a73346ULL, \
    0x1ff7327017aa2a6eULL, 0x594e29c42473d06bULL, 0xf6f31db1899b12d5ULL, 0xc02ac5e47312d3caULL, \
    0xe70201e960cb78b8ULL, 0x6f90ff3b6a65f108ULL, 0x42747a7245e7fa84ULL, 0xd1f507e43ab749b2ULL, \
    0x1c86d265f15750cdULL, 0x3996ce73dd832c1cULL, 0x8e7fba02983224bdULL, 0xba0dec7103255dd4ULL, \
    0x9e9cbd781628fc5bULL, 0xdae8645996edd6a5ULL, 0xdebe0853b1a1d378ULL, 0xa49229d24d014343ULL, \
    0x7be5b9ffda905e1cULL, 0xa3c95eaec244aa30ULL, 0x0230bca8f4df0544ULL, 0x4135c2bebfe148c6ULL, \
    0x166fc0cc438a3c72ULL, 0x3762b59a8ae83efaULL, 0xe8928a4c89114750ULL, 0x2a440b51a4945ee5ULL, \
    0x80cefd2b7d99ff83ULL, 0xbb9879c6e61fd62aULL, 0x6e7c8f1a84265034ULL, 0x164bb2de1bbeddc8ULL, \
    0xf3c12fe54d5c653bULL, 0x40b9e922ed9771e2ULL, 0x551f5b0fbe7b1840ULL, 0x25032aa7c4cb1811ULL, \
    0xaaed34074b164346ULL, 0x8ffd96bbf9c9c81dULL, 0x70fc91eb5937085cULL, 0x7f795e2a5f915440ULL, \
    0x4543d9df5476d3cbULL, 0xf172d73e004fc90dULL, 0xdfd1c4febcc81238ULL, 0xbc8dfb627fe558fcULL, \


static const uint64_t RC_HOST[ROUNDS * WIDTH] = {QP_POSEIDON_RC_LIST};
__constant__ static const uint64_t RC_DEV[ROUNDS * WIDTH] = {QP_POSEIDON_RC_LIST};
// compile-time view (constants folded into instruction operands)
constexpr uint64_t RC_CX[ROUNDS * WIDTH] = {QP_POSEIDON_RC_LIST};
__host__ __device__ constexpr uint64_t rc_cx(int i) { return RC_CX[i]; }

QP_HD uint64_t rc(int i) {
#ifdef __HIP_DEVICE_COMPILE__
  return RC_DEV[i];
#else
  return RC_HOST[i];
#endif
}

QP_HD uint64_t sbox(uint64_t x) {
  uint64_t x2 = gl::sqr(x);
  uint64_t x3 = gl::mul(x2, x);
  uint64_t x4 = gl::sqr(x2);
  return gl::mul(x3, x4);
}

QP_HD void mds(uint64_t s[WIDTH]) {
  uint64_t o[WIDTH];
#pragma unroll
  for (int r = 0; r < WIDTH; r++) {
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < WIDTH; i++) gl::mac_small(s[(i + r) % WIDTH], mds_circ(i), lo, hi);
    if (r == 0) gl::mac_small(s[0], 8, lo, hi);
    o[r] = gl::reduce_split(lo, hi);
  }
#pragma unroll
  for (int r = 0; r < WIDTH; r++) s[r] = o[r];
}

QP_HD void permute(uint64_t s[WIDTH]) {
#pragma unroll
  for (int r = 0; r < ROUNDS; r++) {
#pragma unroll
    for (int i = 0; i < WIDTH; i++) s[i] = gl::add(s[i], rc(r * WIDTH + i));
    if (r < HALF_FULL || r >= HALF_FULL + PARTIAL) {
#pragma unroll
      for (int i = 0; i < WIDTH; i++) s[i] = sbox(s[i]);
    } else {
      s[0] = sbox(s[0]);
    }
    mds(s);
  }
}

// plonky2 hash_no_pad over a strided column vector (host-side helper form)
QP_HD void two_to_one(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
  uint64_t s[WIDTH] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], 0, 0, 0, 0};
  permute(s);
  out[0] = s[0]; out[1] = s[1]; out[2] = s[2]; out[3] = s[3];
}

}  // namespace ps
