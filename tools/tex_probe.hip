// Probe: which HIP array / image-object creation paths work on this box
// (texture path for the renderer's texels).  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(unsigned long long obj, unsigned *out, int w, int h) {
    int x = threadIdx.x % w, y = threadIdx.x / w;
    if (y >= h) return;
    auto *desc = (unsigned int __attribute__((address_space(4))) *)obj;
    int2 c{x, y};
    auto v = __ockl_image_load_2D(desc, get_native_vector(c));
    out[3 * threadIdx.x + 0] = __float_as_uint(v.x);
    out[3 * threadIdx.x + 1] = __float_as_uint(v.y);
    out[3 * threadIdx.x + 2] = __float_as_uint(v.z);
}
int main() {
    int img = -1, img2w = -1;
    (void)hipDeviceGetAttribute(&img, hipDeviceAttributeImageSupport, 0);
    (void)hipDeviceGetAttribute(&img2w, hipDeviceAttributeMaxTexture2DWidth, 0);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    printf("device %s gcnArch %s imageSupport=%d maxTexture2DWidth=%d\n", prop.name, prop.gcnArchName, img, img2w);
    const int w = 7, h = 5;
    std::vector<unsigned char> rgba(w * h * 4);
    for (int i = 0; i < w * h * 4; i++) rgba[i] = (unsigned char)(i * 37 + 11);
    hipChannelFormatDesc cd = hipCreateChannelDesc(8, 8, 8, 8, hipChannelFormatKindUnsigned);
    for (int variant = 0; variant < 3; variant++) {
        hipArray_t arr = nullptr;
        unsigned flags = variant == 1 ? hipArraySurfaceLoadStore : 0;
        hipError_t e = hipMallocArray(&arr, &cd, w, h, flags);
        printf("variant %d mallocArray(flags=%u): %s\n", variant, flags, hipGetErrorString(e));
        if (e != hipSuccess) { (void)hipGetLastError(); continue; }
        e = hipMemcpy2DToArray(arr, 0, 0, rgba.data(), w * 4, w * 4, h, hipMemcpyHostToDevice);
        printf("  memcpy2DToArray: %s\n", hipGetErrorString(e));
        hipResourceDesc rd{};
        rd.resType = hipResourceTypeArray;
        rd.res.array.array = arr;
        unsigned long long obj = 0;
        if (variant == 2) {
            hipTextureDesc td{};
            td.addressMode[0] = td.addressMode[1] = hipAddressModeClamp;
            td.filterMode = hipFilterModePoint;
            td.readMode = hipReadModeElementType;
            td.normalizedCoords = 0;
            hipTextureObject_t t = 0;
            e = hipCreateTextureObject(&t, &rd, &td, nullptr);
            printf("  createTextureObject: %s\n", hipGetErrorString(e));
            obj = (unsigned long long)t;
        } else {
            hipSurfaceObject_t so = 0;
            e = hipCreateSurfaceObject(&so, &rd);
            printf("  createSurfaceObject: %s\n", hipGetErrorString(e));
            obj = (unsigned long long)so;
        }
        if (e != hipSuccess) continue;
        unsigned *d = nullptr;
        (void)hipMalloc(&d, w * h * 3 * 4);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, obj, d, w, h);
        e = hipDeviceSynchronize();
        printf("  kernel: %s\n", hipGetErrorString(e));
        std::vector<unsigned> o(w * h * 3);
        (void)hipMemcpy(o.data(), d, o.size() * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < w * h; i++)
            for (int c = 0; c < 3; c++) bad += o[3 * i + c] != rgba[4 * i + c];
        printf("  values wrong: %d (first %u %u %u vs %u %u %u)\n", bad, o[0], o[1], o[2], rgba[0], rgba[1], rgba[2]);
    }
    return 0;
}
