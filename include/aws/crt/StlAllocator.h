#pragma once
/*
 * STL allocator over an aws_allocator, so that Aws::Crt::String and Aws::Crt::Vector have the same
 * types (and therefore the same mangled names and layout) as the reference's
 * (include/aws/crt/Types.h:45-53 there: std::basic_string / std::vector with StlAllocator<T>).
 * A caller that links Base64Encode / Base64Decode against a real aws-crt-cpp build sees the same
 * symbols.  Stateful: it remembers the aws_allocator it was made with (ApiAllocator() by default).
 */
#include <aws/crt/Allocator.h>

#include <cstddef>
#include <memory>

namespace Aws
{
namespace Crt
{
    template <typename T> class StlAllocator : public std::allocator<T>
    {
      public:
        using Base = std::allocator<T>;
        using size_type = std::size_t;
        template <typename U> struct rebind
        {
            typedef StlAllocator<U> other;
        };

        StlAllocator() noexcept : Base(), m_allocator(ApiAllocator()) {}
        StlAllocator(Allocator *allocator) noexcept : Base(), m_allocator(allocator) {}
        StlAllocator(const StlAllocator &other) noexcept : Base(other), m_allocator(other.m_allocator) {}
        template <class U> StlAllocator(const StlAllocator<U> &other) noexcept : Base(other), m_allocator(other.m_allocator) {}
        ~StlAllocator() {}

        T *allocate(size_type n, const void * = nullptr)
        {
            void *p = aws_mem_acquire(m_allocator, n * sizeof(T));
            if (!p)
            {
                throw std::bad_alloc();
            }
            return static_cast<T *>(p);
        }
        void deallocate(T *p, size_type) { aws_mem_release(m_allocator, p); }

        Allocator *m_allocator;
    };

    template <typename T, typename U> bool operator==(const StlAllocator<T> &a, const StlAllocator<U> &b) noexcept
    {
        return a.m_allocator == b.m_allocator;
    }
    template <typename T, typename U> bool operator!=(const StlAllocator<T> &a, const StlAllocator<U> &b) noexcept
    {
        return !(a == b);
    }
} // namespace Crt
} // namespace Aws
